#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1; s=$?; echo "gpu tests: $s"; tail -2 gpurun_out/pytest_gpu.log
[ $s -eq 0 ] || exit $s
timeout -k 10 300 python benchmarks/kernel_bench.py > gpurun_out/kernel_bench.log 2>&1 || exit $?
tail -1 gpurun_out/kernel_bench.log
timeout -k 10 600 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 32 > gpurun_out/decode256.log 2>&1 || exit $?
grep '^{' gpurun_out/decode256.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --out gpurun_out/bench_closed.json > gpurun_out/bench_closed.log 2>&1 || exit $?
tail -1 gpurun_out/bench_closed.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --mode wave --out gpurun_out/bench_wave.json > gpurun_out/bench_wave.log 2>&1 || exit $?
tail -1 gpurun_out/bench_wave.log
