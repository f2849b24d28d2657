#!/usr/bin/env bash
# GPU test suite only (kernel numerics, engine, beam search, training on the GPU), one process,
# per-test time limit so a hang names its test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
s=$?
tail -15 gpurun_out/pytest_gpu.log
exit $s
