#!/bin/bash
# Large prefills of mixed step graphs back to back after the decode attention (32x32 kernel,
# NGA_PF_SEQ_MIN work items) vs the 16x16 kernel beside it: engine GPU tests in the new mode,
# then the headline interleaved.
set -o pipefail
O=gpurun_out/r3_pfseq3; mkdir -p $O
export PYTHONUNBUFFERED=1
NGA_PF_SEQ_MIN=640 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $O/test_engine.log 2>&1 || { tail -30 $O/test_engine.log; exit 1; }
tail -1 $O/test_engine.log
for r in 1 2 3; do
  for v in 640 384; do
    NGA_PF_SEQ_MIN=$v timeout -k 10 400 python bench.py --steps 12 --warmup 4 > $O/bench_${v}_r$r.json 2> $O/bench_${v}_r$r.err || { tail -20 $O/bench_${v}_r$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${v}_r$r.json'));print('seq_min=$v', d['value'],d['p50_latency_ms'])"
  done
done
