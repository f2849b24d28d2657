#!/usr/bin/env bash
# Round-2 baseline on a fresh box: GPU tests, smoke, headline bench, kernel-level profile.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r2_base"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 $O/pytest_gpu.log
[ $s -ne 0 ] && exit $s
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -1 $O/smoke.log
[ $s -ne 0 ] && exit $s
timeout -k 10 420 python bench.py --steps 5 --warmup 2 --out $O/bench.json > $O/bench.log 2>&1
s=$?; echo "bench exit $s"; cat $O/bench.json
[ $s -ne 0 ] && exit $s
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw_bench" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 > "$O/prof_bench.log" 2>&1
s=$?; echo "prof exit $s"
python3 "$R/scripts/summarize_prof.py" "$O/raw_bench" > "$O/bench_kernels.txt" 2>&1
head -30 "$O/bench_kernels.txt"
rm -rf "$O/raw_bench"
exit $s
