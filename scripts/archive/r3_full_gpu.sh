#!/usr/bin/env bash
# Whole GPU test suite (one pytest process), smoke(), then the headline kernel profile.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
O="$R/gpurun_out/${1:-r3_full}"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
[ -n "${SKIP_PROF:-}" ] && exit 0
bash "$R/scripts/r3_prof.sh" "${1:-r3_full}_prof"
