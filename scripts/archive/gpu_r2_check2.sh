#!/usr/bin/env bash
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=r2_check2 bash scripts/gpu_r2_check.sh || exit $?
O="$R/gpurun_out/r2_check2"
timeout -k 10 600 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 --out $O/bench_mixtral.json > $O/bench_mixtral.log 2>&1
s=$?; echo "mixtral bench exit $s"; cat $O/bench_mixtral.json
exit $s
