#!/bin/bash
# Round 5: weight-in-registers decode GEMM (gemm_wreg.hip) numerics + sweep against the LDS tiles
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_wreg
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "skinny_gemm_every_cfg" > $out/test.txt 2>&1 || { tail -40 $out/test.txt; exit 1; }
tail -3 $out/test.txt
timeout -k 10 600 python -u benchmarks/skinny_gemm.py --check --all --ms 256,128,64 --shapes gate_up,o,down,qkv > $out/sweep.jsonl 2>&1
rc=$?
grep '"best_gemm"' $out/sweep.jsonl | cut -c1-400
exit $rc
