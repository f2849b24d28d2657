#!/bin/bash
# Round 6: the whole GPU test suite (every failure listed)
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_suite}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf -s > $out/pytest_gpu.log 2>&1
rc=$?
grep -E "teacher-forced rows|greedy smoke" $out/pytest_gpu.log | tail -8
tail -4 $out/pytest_gpu.log
exit $rc
