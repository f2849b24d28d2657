#!/usr/bin/env bash
# Kernel-time breakdown of the headline bench (rocprofv3 --kernel-trace --stats; graph-
# replayed kernels included); only the summary is kept.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r3_prof}"
shift || true
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw" -o run -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 "$@" > "$O/bench.log" 2>&1
s=$?
grep '^{' "$O/bench.log" | tail -1 > "$O/bench.json"
python3 "$R/scripts/summarize_prof.py" "$O/raw" > "$O/kernels.txt" 2>&1
python3 "$R/scripts/attn_overlap.py" "$O/raw" > "$O/attn_overlap.json" 2>&1
rm -rf "$O/raw"
exit $s
