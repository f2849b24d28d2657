#!/bin/bash
# Round 6: mixed-step prefill budget (--mixed-prefill-tokens) with the no-short-tail alignment,
# interleaved on one box: headline (8 steps)
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_budget}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for i in 1 2; do
  for b in 4096 3072 5120; do
    timeout -k 10 400 python bench.py --steps 8 --warmup 2 --mixed-prefill-tokens $b > $out/bench_m${b}_$i.json 2> $out/bench_m${b}_$i.err || { tail -20 $out/bench_m${b}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_m${b}_$i.json'));sg=d['step_graphs'];print('budget=$b', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'], sg['captured_in_timed_region'])"
  done
done
