#!/usr/bin/env bash
# Kernel trace (+ ROCTx markers) of a short closed-loop bench; keeps only the gap analysis.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/gaps"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
export NGA_MARKERS=1
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$O/raw" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 > "$O/bench.log" 2>&1
s=$?
echo "bench exit $s"; grep '^{' "$O/bench.log" | cut -c1-200
python3 "$R/scripts/gap_analysis.py" "$O/raw" > "$O/gaps.txt" 2>&1
head -45 "$O/gaps.txt"
rm -rf "$O/raw"
exit $s
