#!/bin/bash
# Round 6: TP = 8 rehearsal tests, the TP = 8 agent A/B, then the BK = 32 GEMM tile sweep
set -o pipefail
cd "$(dirname "$0")/../../.."
bash scripts/archive/r6/tp8.sh r6_tp8 ; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/archive/r6/tp8_agent.sh r6_tp8_agent || exit $?
bash scripts/archive/r6/bk32.sh r6_bk32
