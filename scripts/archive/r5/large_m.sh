#!/bin/bash
# Round 5: the decode-shape GEMM's large tiles at the mixed-step M (4,096 prefill + 256 decode
# rows) against the library GEMM (+ silu_mul for gate/up): is a hand-written MFMA kernel with
# the SwiGLU epilogue in reach of the library at this M?
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_large_m
mkdir -p $out
: > $out/sweep.jsonl
for s in gate_up down o qkv; do
  timeout -k 10 150 python -u benchmarks/skinny_gemm.py --shapes $s --ms 4352 --cfgs 0,4,12,13,14,16 --iters 20 --all --check >> $out/sweep.jsonl 2>&1 || { tail -20 $out/sweep.jsonl; exit 1; }
done
cat $out/sweep.jsonl
