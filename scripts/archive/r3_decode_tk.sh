#!/usr/bin/env bash
# Decode attention in-launch partition combine: numerics tests, kernel A/B (tickets vs the
# separate combine kernel), then the FP8 W8A8 + FP8-KV headline run (host launch vs wait).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r3_tk}"
mkdir -p "$O"
cd "$R"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "decode" --timeout 120 --timeout-method thread > "$O/test_decode.log" 2>&1 || { tail -30 "$O/test_decode.log"; exit 1; }
tail -2 "$O/test_decode.log"
timeout -k 10 300 python benchmarks/kernel_bench.py --only decode > "$O/kb_decode_tickets.json" 2> "$O/kb.err" || exit 1
NGA_DECODE_TICKETS=0 timeout -k 10 300 python benchmarks/kernel_bench.py --only decode > "$O/kb_decode_combine_kernel.json" 2>> "$O/kb.err" || exit 1
[ -n "${SKIP_FP8:-}" ] && exit 0
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --fp8 --kv-fp8 > "$O/bench_fp8.json" 2> "$O/bench_fp8.err" || exit 1
