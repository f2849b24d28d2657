#!/bin/bash
# Round 4: skinny GEMM in the model: numerics tests, qkv table row with the RoPE consumer,
# decode-step A/B (library vs skinny)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_integrate; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "skinny or splitk or rope" > $O/kern.txt 2>&1 || { tail -30 $O/kern.txt; exit 1; }
tail -2 $O/kern.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "skinny or gqa or step_graphs or forward_matches or graph_decode" > $O/engine.txt 2>&1 || { tail -40 $O/engine.txt; exit 1; }
grep -E "PASSED|FAILED" $O/engine.txt
timeout -k 10 300 python -u benchmarks/skinny_table.py --shapes qkv --merge nv_genai_amd/assets/skinny_gemm_gfx950.json --out $O/skinny_gemm_gfx950.json > $O/qkv_table.jsonl 2>&1 || { tail -5 $O/qkv_table.jsonl; exit 1; }
cut -c1-200 $O/qkv_table.jsonl | grep shape
for v in 0 1; do
  NGA_SKINNY=$v timeout -k 10 300 python -u benchmarks/decode_step.py --batch 256 --ctx 1350 --steps 32 > $O/decode_skinny$v.json 2> $O/decode_skinny$v.err || { tail -20 $O/decode_skinny$v.err; exit 1; }
  echo "skinny=$v $(cat $O/decode_skinny$v.json)"
done
