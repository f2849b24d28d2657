#!/bin/bash
# Submit-path sync probe + the 2-rank bench rehearsal tests on the 1-GPU box.
set -o pipefail
O=gpurun_out/r3_probe1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python benchmarks/submit_probe.py > $O/submit_probe.json 2> $O/submit_probe.err || { tail -20 $O/submit_probe.err; exit 1; }
cat $O/submit_probe.json
timeout -k 10 600 python -u -m pytest tests/test_bench_multirank_gpu.py -x -v --timeout 280 --timeout-method thread > $O/multirank.log 2>&1 || { tail -40 $O/multirank.log; exit 1; }
tail -3 $O/multirank.log
bash scripts/r3_prof.sh r3_probe1_prof && cat gpurun_out/r3_probe1_prof/attn_overlap.json
