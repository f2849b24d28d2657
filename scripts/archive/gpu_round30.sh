#!/usr/bin/env bash
# Kernel profile of the FP8 W8A8 headline workload.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r30"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --fp8 > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
python3 "$R/scripts/summarize_prof.py" "$O/raw" > "$O/fp8_kernels.txt" 2>&1
rm -rf "$O/raw"
head -24 "$O/fp8_kernels.txt" | cut -c1-200
tail -3 "$O/fp8_kernels.txt"
