#!/bin/bash
# Half-page ring form of the LDS-DMA decode kernel (NGA_DECODE_DMA=2): decode numerics tests for
# both forms, then the kernel bench (forms interleaved).
set -o pipefail
O=gpurun_out/r3_ring; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_families_gpu.py -k "decode_attention" -x -v --timeout 120 --timeout-method thread > $O/test_decode.log 2>&1 || { grep -n "Error\|assert\|FAIL" $O/test_decode.log | head -20; tail -5 $O/test_decode.log; exit 1; }
tail -2 $O/test_decode.log
timeout -k 10 400 python benchmarks/kernel_bench.py --only decode > $O/kb_decode.json 2> $O/kb_decode.err || { tail -20 $O/kb_decode.err; exit 1; }
python -c "import json;d=json.load(open('$O/kb_decode.json'));[print(k,v) for k,v in d.items() if 'forms' in k]"
