#!/bin/bash
# Round 4: weight-streaming GEMV (M <= 4): numerics tests, then GEMV vs skinny vs library
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_gemv; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "gemv" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
timeout -k 10 300 python -u benchmarks/gemv_bench.py > $O/gemv.jsonl 2> $O/gemv.err || { tail -20 $O/gemv.err; exit 1; }
cat $O/gemv.jsonl
