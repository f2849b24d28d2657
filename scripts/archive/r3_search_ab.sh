#!/bin/bash
# Search kernel tests + bench (LDS-DMA vs register form), then the submit-path A/B.
set -o pipefail
O=gpurun_out/r3_search_dma; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_search_gpu.py -x -v --timeout 200 --timeout-method thread > $O/test_search.log 2>&1 || { grep -n "Error\|assert" $O/test_search.log | head -20; tail -5 $O/test_search.log; exit 1; }
tail -2 $O/test_search.log
timeout -k 10 400 python benchmarks/kernel_bench.py --only search > $O/kb_search.json 2> $O/kb_search.err || { tail -20 $O/kb_search.err; exit 1; }
cat $O/kb_search.json
bash scripts/r3_ab_submit.sh
timeout -k 10 300 python benchmarks/kernel_bench.py --only decode_small > $O/kb_decode_small.json 2> $O/kb_decode_small.err || { tail -20 $O/kb_decode_small.err; exit 1; }
cat $O/kb_decode_small.json
