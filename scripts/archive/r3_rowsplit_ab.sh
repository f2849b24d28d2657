#!/bin/bash
# Row-split o / down GEMMs (NGA_ROW_SPLIT): gate/up probe, engine GPU tests, then the headline
# interleaved on one box (split on / off twice).
set -o pipefail
O=gpurun_out/r3_rowsplit; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python benchmarks/row_split_gemm.py --only gate_up --ms 4352 > $O/probe_gate_up.jsonl 2> $O/probe_gate_up.err || { tail -5 $O/probe_gate_up.err; exit 1; }
cat $O/probe_gate_up.jsonl
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $O/test_engine.log 2>&1 || { tail -30 $O/test_engine.log; exit 1; }
tail -1 $O/test_engine.log
for r in 1 2; do
  for v in 1 0; do
    NGA_ROW_SPLIT=$v timeout -k 10 400 python bench.py --steps 12 --warmup 4 > $O/bench_${v}_r$r.json 2> $O/bench_${v}_r$r.err || { tail -20 $O/bench_${v}_r$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${v}_r$r.json'));print('split=$v', d['value'],d['p50_latency_ms'])"
  done
done
