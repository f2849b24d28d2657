#!/usr/bin/env bash
# Kernel profile of the closed-loop bench (mixed steps) + DSP kernel tests.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider -rf -k "dsp or fir or demod or resample or mining" > gpurun_out/pytest_dsp.log 2>&1; echo "dsp tests $?"; tail -3 gpurun_out/pytest_dsp.log
PROFS="run bench_closed 900 python3 $R/bench.py --steps 1 --warmup 1" bash scripts/gpu_prof_one.sh
