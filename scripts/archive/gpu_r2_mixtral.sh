#!/usr/bin/env bash
# Mixtral-8x7B (the reference's default chat model) on the headline RAG workload, plus a
# kernel profile of a short run.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r2_mixtral"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 --out $O/bench_mixtral.json > $O/bench_mixtral.log 2>&1
s=$?; echo "bench exit $s"; tail -3 $O/bench_mixtral.log
[ $s -ne 0 ] && exit $s
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw" -o run -- python3 "$R/bench.py" --model mixtral-8x7b --steps 1 --warmup 1 --concurrency 128 > "$O/prof.log" 2>&1
s=$?; echo "prof exit $s"
python3 "$R/scripts/summarize_prof.py" "$O/raw" > "$O/kernels.txt" 2>&1
head -25 "$O/kernels.txt"
rm -rf "$O/raw"
exit $s
