#!/bin/bash
# Decode attention with the per-CU split for the LDS-DMA kernel at every batch size:
# kernel + engine tests, decode kernel benches.
set -o pipefail
O=gpurun_out/r3_decode_small; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_families_gpu.py -x -v --timeout 200 --timeout-method thread -k "decode or window or fp8" > $O/test_decode.log 2>&1 || { grep -n "Error\|assert" $O/test_decode.log | head -20; tail -5 $O/test_decode.log; exit 1; }
tail -2 $O/test_decode.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread > $O/test_engine.log 2>&1 || { grep -n "Error\|assert" $O/test_engine.log | head -20; tail -5 $O/test_engine.log; exit 1; }
tail -2 $O/test_engine.log
timeout -k 10 300 python benchmarks/kernel_bench.py --only decode_small > $O/kb_decode_small.json 2> $O/kb_decode_small.err || { tail -20 $O/kb_decode_small.err; exit 1; }
cat $O/kb_decode_small.json
timeout -k 10 300 python benchmarks/kernel_bench.py --only decode > $O/kb_decode.json 2> $O/kb_decode.err || { tail -20 $O/kb_decode.err; exit 1; }
cat $O/kb_decode.json
