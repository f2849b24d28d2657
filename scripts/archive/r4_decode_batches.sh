#!/bin/bash
# Round 4: decode step latency at small and serving batches, decode-shape GEMM off / on
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_decode_batches; mkdir -p $O
for b in 1 16 64 128 256; do
  for sk in 0 1; do
    NGA_SKINNY=$sk timeout -k 10 240 python -u benchmarks/decode_step.py --batch $b --ctx 1350 > $O/b${b}_sk$sk.json 2> $O/b${b}_sk$sk.err || { tail -10 $O/b${b}_sk$sk.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b${b}_sk$sk.json'));print('batch $b skinny $sk', d['step_ms'], d['eff_TBps'])"
  done
done
