#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider -rf -k "sample" > gpurun_out/pytest_sample.log 2>&1; s=$?; echo "sample tests $s"; tail -3 gpurun_out/pytest_sample.log
[ $s -eq 0 ] || exit $s
for n in 1 2; do
  NGA_PREFILL_NCG=$n timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -p no:cacheprovider -rf -k "prefill or attention or forward or chunked" > gpurun_out/pytest_prefill_ncg$n.log 2>&1; s=$?; echo "prefill tests ncg=$n: $s"; tail -2 gpurun_out/pytest_prefill_ncg$n.log
  [ $s -eq 0 ] || exit $s
  NGA_PREFILL_NCG=$n timeout -k 10 300 python benchmarks/kernel_bench.py > gpurun_out/kernel_bench_ncg$n.log 2>&1 || exit $?
  tail -1 gpurun_out/kernel_bench_ncg$n.log
done
