#!/usr/bin/env bash
# Measure with the shipped GEMM table: decode-step micro-bench, full bench, kernel profile.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 600 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 32 > gpurun_out/decode256.log 2>&1 || exit $?
grep '^{' gpurun_out/decode256.log
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --out gpurun_out/bench_c256.json > gpurun_out/bench_c256.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c256.log
PROFS="run decode256 600 python3 $R/benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16" bash scripts/gpu_prof_one.sh
