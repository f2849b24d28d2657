#!/bin/bash
# Round 5: numerics evidence + the whole GPU suite, then the large-M GEMM probe
set -o pipefail
cd "$(dirname "$0")/../.."
bash scripts/archive/r5/numerics.sh
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc    # anything but test failures: stop here
bash scripts/archive/r5/large_m.sh | tail -30 || exit 1
mkdir -p gpurun_out/r5_overlap
timeout -k 10 300 python -u benchmarks/overlap_probe.py > gpurun_out/r5_overlap/probe.jsonl 2>&1; r2=$?
cat gpurun_out/r5_overlap/probe.jsonl | tail -5
[ $r2 -eq 0 ] || exit $r2
exit $rc
