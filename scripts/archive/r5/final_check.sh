#!/bin/bash
# Round 5: what the driver runs at round end, on this tree: the GPU suite, then smoke()
set -o pipefail
cd "$(dirname "$0")/../.."
bash scripts/archive/r5/full.sh r5_final_check || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_final_check/smoke.txt 2>&1 || { tail -20 gpurun_out/r5_final_check/smoke.txt; exit 1; }
tail -2 gpurun_out/r5_final_check/smoke.txt
