#!/bin/bash
# Round 5: the whole GPU test suite (every failure listed), then the headline script
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/${1:-r5_full}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $out/pytest_gpu.log 2>&1
rc=$?
tail -25 $out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc    # 1 = test failures (read them); anything else: stop
if [ "${2:-}" = "headline" ]; then bash scripts/archive/r5/headline.sh ${1:-r5_full}_headline; fi
exit $rc
