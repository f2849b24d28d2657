#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 32 > gpurun_out/decode256.log 2>&1 || exit $?
grep '^{' gpurun_out/decode256.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --out gpurun_out/bench_closed.json > gpurun_out/bench_closed.log 2>&1 || exit $?
tail -1 gpurun_out/bench_closed.log | cut -c1-200
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --mode wave --out gpurun_out/bench_wave.json > gpurun_out/bench_wave.log 2>&1 || exit $?
tail -1 gpurun_out/bench_wave.log | cut -c1-200
