#!/bin/bash
# 2-rank bench rehearsal tests on the 1-GPU box, a headline run with the submit-path
# breakdown, then the headline kernel trace with the mixed-step attention overlap analysis.
set -o pipefail
O=gpurun_out/r3_probe1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_bench_multirank_gpu.py -x -v --timeout 280 --timeout-method thread > $O/multirank.log 2>&1 || { grep -n "Error" $O/multirank.log | head -20; tail -5 $O/multirank.log; exit 1; }
tail -3 $O/multirank.log
timeout -k 10 400 python bench.py --steps 8 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['submit_host_ms'],d['host_work_ms'],d['host_s'])"
bash scripts/r3_prof.sh r3_probe1_prof && cat gpurun_out/r3_probe1_prof/attn_overlap.json
