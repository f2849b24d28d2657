#!/bin/bash
# Round 4: skinny GEMM numerics + sweep
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4_skinny
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "skinny or splitk" > gpurun_out/r4_skinny/test.txt 2>&1 || { tail -30 gpurun_out/r4_skinny/test.txt; exit 1; }
tail -3 gpurun_out/r4_skinny/test.txt
timeout -k 10 600 python -u benchmarks/skinny_gemm.py --check --ms 64,128,256,512 > gpurun_out/r4_skinny/sweep.jsonl 2>&1
rc=$?
tail -25 gpurun_out/r4_skinny/sweep.jsonl
exit $rc
