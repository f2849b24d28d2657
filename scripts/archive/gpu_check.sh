#!/usr/bin/env bash
# GPU-box validation: kernel numerics + engine tests, smoke(), then a short bench.
# Each GPU step has its own time limit; a crash/abort/timeout ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1
s=$?
echo "pytest exit $s"; tail -5 gpurun_out/pytest_gpu.log
if [ $s -ne 0 ] && [ $s -ne 1 ]; then exit $s; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -3 gpurun_out/smoke.log
if [ $s -ne 0 ]; then exit $s; fi
timeout -k 10 ${BENCH_TIMEOUT:-900} python bench.py ${BENCH_ARGS:---steps 2 --warmup 1} --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1
s=$?; echo "bench exit $s"; tail -3 gpurun_out/bench.log
exit $s
