#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python benchmarks/gemm_sweep.py > gpurun_out/gemm_sweep_default.log 2>&1 || exit $?
cat gpurun_out/gemm_sweep_default.log
timeout -k 10 300 python benchmarks/gemm_sweep.py --tuned > gpurun_out/gemm_sweep_tuned.log 2>&1 || exit $?
cat gpurun_out/gemm_sweep_tuned.log
