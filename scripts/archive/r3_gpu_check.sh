#!/bin/bash
# Round-3 GPU check: kernel numerics, engine (incl. step graphs), custom all-reduce at 4
# ranks, kernel benches, a short headline bench. Every GPU step has its own time limit and
# the chain stops at the first failure.
set -o pipefail
OUT=${1:-gpurun_out/r3_check}
mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 420 python -u -m pytest tests/test_kernels_gpu.py tests/test_search_gpu.py -x -v --timeout 200 --timeout-method thread > "$OUT/kernels.log" 2>&1 &&
timeout -k 10 420 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread > "$OUT/engine.log" 2>&1 || exit 1
fi

timeout -k 10 300 python -u -m pytest tests/test_custom_ar_gpu.py -x -v --timeout 200 --timeout-method thread > "$OUT/custom_ar.log" 2>&1 &&
timeout -k 10 200 python benchmarks/kernel_bench.py --only bw > "$OUT/kb_bw.json" 2> "$OUT/kb_bw.err" &&
timeout -k 10 300 python benchmarks/kernel_bench.py --only prefill > "$OUT/kb_prefill.json" 2> "$OUT/kb_prefill.err" &&
timeout -k 10 300 python benchmarks/kernel_bench.py --only decode > "$OUT/kb_decode.json" 2> "$OUT/kb_decode.err" &&
NGA_DECODE_NT=1 timeout -k 10 300 python benchmarks/kernel_bench.py --only decode > "$OUT/kb_decode_nt.json" 2> "$OUT/kb_decode_nt.err" &&
timeout -k 10 300 python benchmarks/kernel_bench.py --only search > "$OUT/kb_search.json" 2> "$OUT/kb_search.err" &&
timeout -k 10 500 python bench.py --steps 5 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
