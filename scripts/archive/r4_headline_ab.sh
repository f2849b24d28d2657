#!/bin/bash
# Round 4: headline bench A/B, skinny decode-shape GEMMs off / on (interleaved: off, on, on, off)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_headline_ab; mkdir -p $O
i=0
for v in 0 1 1 0; do
  i=$((i+1))
  NGA_SKINNY=$v timeout -k 10 420 python -u bench.py --steps 10 --warmup 3 > $O/bench_${i}_skinny$v.json 2> $O/bench_${i}_skinny$v.err || { tail -20 $O/bench_${i}_skinny$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_${i}_skinny$v.json'));print('skinny=$v', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'])"
done
timeout -k 10 300 python -u benchmarks/skinny_gemm.py --ms 64,256 --shapes o,qkv,down,gate_up --cfgs 1,2,3,10,12,13,16,17,18,19,20,21,22,23 --all > $O/sweep_il.jsonl 2>&1 || { tail -20 $O/sweep_il.jsonl; exit 1; }
grep '"lib_us"' $O/sweep_il.jsonl | cut -c1-330
