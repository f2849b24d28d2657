#!/usr/bin/env bash
# Full GPU validation of the current tree, then a concurrency sweep of the headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r36; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 $O/pytest_gpu.log
if [ $s -ne 0 ] && [ $s -ne 1 ]; then exit $s; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -2 $O/smoke.log
[ $s -ne 0 ] && exit $s
for c in 256 384 512; do
  timeout -k 10 420 python bench.py --steps 2 --warmup 1 --concurrency $c --out $O/bench_c$c.json > $O/bench_c$c.log 2>&1
  s=$?; echo "bench c=$c exit $s"; cat $O/bench_c$c.json
  [ $s -ne 0 ] && exit $s
done
exit 0
