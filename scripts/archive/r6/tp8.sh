#!/bin/bash
# Round 6: the TP = 8 one-GPU rehearsal tests (8 ranks on cuda:0)
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_tp8}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_tp8_rehearsal_gpu.py -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $out/pytest_tp8.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error" $out/pytest_tp8.log | tail -20
tail -5 $out/pytest_tp8.log
exit $rc
