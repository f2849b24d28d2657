#!/usr/bin/env bash
# Validation + profile of the current tree: GPU tests, headline bench, rocprofv3 kernel stats
# of the default (256-client closed-loop) bench. Each GPU step has its own limit; the first
# failure ends the script.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r21"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread -rf > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --out "$O/bench.json" > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw_bench" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
python3 "$R/scripts/summarize_prof.py" "$O/raw_bench" > "$O/bench_kernels.txt" 2>&1
rm -rf "$O/raw_bench"
head -30 "$O/bench_kernels.txt"
tail -4 "$O/bench_kernels.txt"
