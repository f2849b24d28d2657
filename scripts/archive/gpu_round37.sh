#!/usr/bin/env bash
# Kernel profile of the default headline bench (256 clients) on the rebuilt tree; keeps only
# the summary (the raw kernel trace of a full bench is > 64 MiB).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r38"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 > "$O/bench_prof.log" 2>&1
s=$?; echo "prof exit $s"; grep '^{' "$O/bench_prof.log" | tail -1
python3 "$R/scripts/summarize_prof.py" "$O/raw" > "$O/bench_c256_kernels.txt" 2>&1
rm -rf "$O/raw"
head -30 "$O/bench_c256_kernels.txt"; tail -4 "$O/bench_c256_kernels.txt"
exit $s
