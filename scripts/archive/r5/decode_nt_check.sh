#!/bin/bash
# Round 5: decode_nt default 2 (nt for bf16 pages only): register-kernel numerics, fp8 KV tests,
# then the bf16 decode step on the register kernel at the new default vs 0
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_decode_nt_check
mkdir -p $out
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_kv_fp8.py -m gpu -k "decode or fp8" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for r in 1 2; do
  for v in 2 0; do
    NGA_DECODE_DMA=0 NGA_DECODE_NT=$v timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 48 > $out/decode_reg_${v}_$r.json 2> $out/decode_reg_${v}_$r.err || { tail -5 $out/decode_reg_${v}_$r.err; exit 1; }
    echo "decode (register kernel) decode_nt $v round $r $(python3 -c "import json;d=json.load(open('$out/decode_reg_${v}_$r.json'));print(d['replay_ms'], d['step_ms'])")"
  done
done
