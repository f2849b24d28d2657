#!/usr/bin/env bash
# Embedding rate vs the reference's published encode rate; full GPU suite; kernel profile of
# the headline bench with concurrent mixed-step attention.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r27"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python benchmarks/embed_rate.py --out "$O/embed_rate.json" > "$O/embed_rate.log" 2>&1 || { tail -20 "$O/embed_rate.log"; exit 1; }
cat "$O/embed_rate.json"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread -rf > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw_bench" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
python3 "$R/scripts/summarize_prof.py" "$O/raw_bench" > "$O/bench_kernels.txt" 2>&1
rm -rf "$O/raw_bench"
head -16 "$O/bench_kernels.txt"
tail -3 "$O/bench_kernels.txt"
