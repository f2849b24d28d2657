#!/bin/bash
# Round 5: pipelined TP=2 with step graphs on one GPU + the custom collectives
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_tp
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py tests/test_custom_ar_gpu.py > $out/tests.txt 2>&1
rc=$?
tail -30 $out/tests.txt
exit $rc
