#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1; s=$?; echo "gpu tests: $s"; tail -2 gpurun_out/pytest_gpu.log
[ $s -eq 0 ] || exit $s
timeout -k 10 300 python benchmarks/kernel_bench.py > gpurun_out/kernel_bench.log 2>&1 || exit $?
tail -1 gpurun_out/kernel_bench.log
bash scripts/gpu_pmc_prefill.sh > /dev/null 2>&1; cat gpurun_out/pmc/summary.txt
