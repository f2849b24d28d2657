#!/usr/bin/env bash
# GPU tests (mixed steps), then the closed-loop bench (mixed on/off) and the wave bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -4 gpurun_out/pytest_gpu.log
if [ $s -ne 0 ] && [ $s -ne 1 ]; then exit $s; fi
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --out gpurun_out/bench_closed.json > gpurun_out/bench_closed.log 2>&1 || exit $?
tail -1 gpurun_out/bench_closed.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --mixed-prefill-tokens 0 --out gpurun_out/bench_closed_nomix.json > gpurun_out/bench_closed_nomix.log 2>&1 || exit $?
tail -1 gpurun_out/bench_closed_nomix.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --mode wave --out gpurun_out/bench_wave.json > gpurun_out/bench_wave.log 2>&1 || exit $?
tail -1 gpurun_out/bench_wave.log
