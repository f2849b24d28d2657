#!/usr/bin/env bash
# Tiled RoPE + KV-write kernel: numerics, micro-benchmark, headline bench, multi-turn bench.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r25"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python benchmarks/kernel_bench.py --only rope > "$O/rope.log" 2>&1 || { tail -20 "$O/rope.log"; exit 1; }
grep '^{' "$O/rope.log"
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --out "$O/bench.json" > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-250
timeout -k 10 600 python benchmarks/multi_turn.py --sessions 64 --turns 4 --out "$O/multi_turn_s64.json" \
    > "$O/multi_turn_s64.log" 2>&1 || { tail -20 "$O/multi_turn_s64.log"; exit 1; }
cat "$O/multi_turn_s64.json"
