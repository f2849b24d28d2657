#!/usr/bin/env bash
# Re-validate a freshly rebuilt tree: GPU tests, smoke, default headline bench, kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r37; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 $O/pytest_gpu.log
if [ $s -ne 0 ] && [ $s -ne 1 ]; then exit $s; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -2 $O/smoke.log
[ $s -ne 0 ] && exit $s
timeout -k 10 420 python bench.py --out $O/bench_default.json > $O/bench_default.log 2>&1
s=$?; echo "bench exit $s"; cat $O/bench_default.json
[ $s -ne 0 ] && exit $s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 480 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 1 > $O/prof.log 2>&1
s=$?; echo "prof exit $s"
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -r head -25
exit 0
