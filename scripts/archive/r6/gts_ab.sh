#!/bin/bash
# Round 6: step-graph token bucket granularity (--graph-token-step 256 default vs 128) with the
# no-short-tail alignment, interleaved on one box: headline (8 steps)
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_gts}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for i in 1 2; do
  for g in 256 128; do
    timeout -k 10 400 python bench.py --steps 8 --warmup 2 --graph-token-step $g > $out/bench_g${g}_$i.json 2> $out/bench_g${g}_$i.err || { tail -20 $out/bench_g${g}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_g${g}_$i.json'));sg=d['step_graphs'];print('gts=$g', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'], sg['captured_total'], sg['captured_in_timed_region'], sg['capture_s_in_timed_region'])"
  done
done
