#!/usr/bin/env bash
# Prefill attention with mask-free unmasked tiles + packed softmax VALU: numerics (GPU tests),
# kernel timing, then the headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r39; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 $O/pytest_gpu.log
[ $s -ne 0 ] && exit $s
timeout -k 10 300 python benchmarks/kernel_bench.py --only prefill > $O/kbench_prefill.log 2>&1
s=$?; echo "kbench exit $s"; tail -1 $O/kbench_prefill.log
[ $s -ne 0 ] && exit $s
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s"; tail -1 $O/smoke.log
[ $s -ne 0 ] && exit $s
timeout -k 10 420 python bench.py --out $O/bench_default.json > $O/bench_default.log 2>&1
s=$?; echo "bench exit $s"; cat $O/bench_default.json
exit $s
