#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -p no:cacheprovider -rf -k "prefill or attention or forward or chunked or encoder or mixed" > gpurun_out/pytest_prefill.log 2>&1; s=$?; echo "prefill tests: $s"; tail -2 gpurun_out/pytest_prefill.log
[ $s -eq 0 ] || exit $s
timeout -k 10 300 python benchmarks/kernel_bench.py --only prefill > gpurun_out/kernel_bench.log 2>&1 || exit $?
tail -1 gpurun_out/kernel_bench.log
bash scripts/gpu_pmc_prefill.sh > /dev/null 2>&1; cat gpurun_out/pmc/summary.txt
