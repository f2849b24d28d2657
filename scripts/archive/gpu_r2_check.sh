#!/usr/bin/env bash
# Full GPU suite + smoke + a short headline bench of the current tree.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/${TAG:-r2_check}"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -15
[ $s -ne 0 ] && exit $s
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -1 $O/smoke.log
[ $s -ne 0 ] && exit $s
timeout -k 10 420 python bench.py --steps 3 --warmup 1 --out $O/bench.json > $O/bench.log 2>&1
s=$?; echo "bench exit $s"; cat $O/bench.json
exit $s
