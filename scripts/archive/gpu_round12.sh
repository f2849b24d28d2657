#!/usr/bin/env bash
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --out gpurun_out/bench_closed_rb8.json > gpurun_out/bench_closed_rb8.log 2>&1 || exit $?
tail -1 gpurun_out/bench_closed_rb8.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --retrieval-batch 1 --out gpurun_out/bench_closed_rb1.json > gpurun_out/bench_closed_rb1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_closed_rb1.log
PROFS="run bench_closed 900 python3 $R/bench.py --steps 1 --warmup 1" bash scripts/gpu_prof_one.sh
