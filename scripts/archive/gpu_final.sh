#!/usr/bin/env bash
# Final check of the committed tree: GPU tests and smoke only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -2 $O/pytest_gpu.log
[ $s -ne 0 ] && exit $s
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -1 $O/smoke.log
exit $s
