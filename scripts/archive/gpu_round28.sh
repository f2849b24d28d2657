#!/usr/bin/env bash
# FP8 W8A8 serving mode: kernel + engine numerics, then the headline bench in fp8 (reported
# separately; the headline stays bf16).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r28"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread -k "fp8" > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --fp8 --out "$O/bench_fp8.json" > "$O/bench_fp8.log" 2>&1 || { tail -20 "$O/bench_fp8.log"; exit 1; }
tail -1 "$O/bench_fp8.log" | cut -c1-300
