#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -4 gpurun_out/pytest_gpu.log
if [ $s -ne 0 ] && [ $s -ne 1 ]; then exit $s; fi
timeout -k 10 600 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 32 > gpurun_out/decode256.log 2>&1 || exit $?
grep '^{' gpurun_out/decode256.log
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --concurrency 256 --out gpurun_out/bench_c256.json > gpurun_out/bench_c256.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c256.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=10 \
  timeout -k 10 900 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 32 > gpurun_out/decode256_tuned.log 2>&1
s=$?; echo "tuned exit $s"; grep '^{' gpurun_out/decode256_tuned.log; tail -3 gpurun_out/decode256_tuned.log
ls -la gpurun_out/
exit 0
