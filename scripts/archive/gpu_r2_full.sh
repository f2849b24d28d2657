#!/usr/bin/env bash
# Full GPU suite + smoke (what the driver runs at round end)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
O="$R/gpurun_out/r2_full${TAG:+_$TAG}"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -5 $O/pytest_gpu.log; [ $s -ne 0 ] && exit $s
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -2 $O/smoke.log; exit $s
