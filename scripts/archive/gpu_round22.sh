#!/usr/bin/env bash
# Decode-attention split change: kernel numerics, decode micro-benchmark, headline bench.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r22"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python benchmarks/kernel_bench.py --only decode > "$O/decode.log" 2>&1 || { tail -20 "$O/decode.log"; exit 1; }
grep '^{' "$O/decode.log"
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --out "$O/bench.json" > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-260
