#!/bin/bash
# Round 4: kernel table of the decode-only step (256 x 1,350, llama3-8b, graph replay)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r4_prof_decode"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw" -o run -- \
  python3 "$R/benchmarks/decode_step.py" --batch ${B:-256} --ctx 1350 > "$O/decode.log" 2>&1
s=$?
python3 "$R/scripts/summarize_prof.py" "$O/raw" > "$O/kernels.txt" 2>&1
rm -rf "$O/raw"
head -40 "$O/kernels.txt"
exit $s
