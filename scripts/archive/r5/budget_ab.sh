#!/bin/bash
# Round 5: mixed-step prefill budget so that prefill + decode rows stay at 4,096 (one library
# GEMM per projection, no row split and no extra 256-row decode-shape pass) vs the shipped
# 4,096 prefill tokens (+ up to 256 decode rows = 4,352). Interleaved, 10 steps / 3 warm-up.
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_budget
mkdir -p $out
for r in 1 2; do
  for b in 4096 3840 3584; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --mixed-prefill-tokens $b > $out/b${b}_$r.json 2> $out/b${b}_$r.err || { tail -20 $out/b${b}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$out/b${b}_$r.json'));print('budget $b round $r', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'], d['steps_prefill_decode_mixed'])"
  done
done
