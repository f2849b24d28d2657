#!/bin/bash
# Round 5: non-temporal 2-byte V^T page stores in the RoPE / KV-write kernels (form rope_vnt):
# numerics, then kernel_bench rope interleaved 0 / 1 / 0 / 1, then the decode step
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_rope_vnt
mkdir -p $out
timeout -k 10 200 python -u -m pytest -q -p no:cacheprovider --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "rope" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for v in 0 1 0 1; do
  NGA_ROPE_VNT=$v timeout -k 10 120 python benchmarks/kernel_bench.py --only rope > $out/kb_$v.txt 2>&1 || { tail -5 $out/kb_$v.txt; exit 1; }
  echo "vnt $v $(tail -1 $out/kb_$v.txt)"
done
for v in 0 1; do
  NGA_ROPE_VNT=$v timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 32 > $out/decode_$v.json 2> $out/decode_$v.err || { tail -5 $out/decode_$v.err; exit 1; }
  echo "decode vnt $v $(tail -1 $out/decode_$v.json)"
done
