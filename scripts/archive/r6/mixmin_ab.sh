#!/bin/bash
# Round 6: accumulate prompt tokens before a mixed step (--mixed-min-tokens, max wait 4 steps)
# with the no-short-tail alignment, interleaved on one box: headline (8 steps)
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_mixmin}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for i in 1 2; do
  for m in 0 2048; do
    timeout -k 10 400 python bench.py --steps 8 --warmup 2 --mixed-min-tokens $m > $out/bench_mm${m}_$i.json 2> $out/bench_mm${m}_$i.err || { tail -20 $out/bench_mm${m}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_mm${m}_$i.json'));print('mixed_min=$m', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'])"
  done
done
