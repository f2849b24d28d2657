#!/bin/bash
# Round 4: TP=2 (two ranks sharing the GPU, custom all-reduce) with and without the decode-shape
# kernel on the rank shards
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_tp_skinny; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py tests/test_engine_gpu.py -m gpu -k "tp2 or skinny_gemm_path" > $O/test.txt 2>&1 || { tail -40 $O/test.txt; exit 1; }
grep -E "PASS|FAIL" $O/test.txt
