#!/usr/bin/env bash
# Model families: new kernel numerics (GPU tests), regression of the Llama kernels, MoE and
# attention micro-benchmarks.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r2_fam"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_families_gpu.py tests/test_kernels_gpu.py -v -p no:cacheprovider -rf --timeout 120 --timeout-method thread > $O/pytest_fam.log 2>&1
s=$?; echo "pytest exit $s"; grep -E "passed|failed|FAILED|Error" $O/pytest_fam.log | tail -15
[ $s -ne 0 ] && exit $s
timeout -k 10 300 python benchmarks/kernel_bench.py --only decode > $O/kb_decode.log 2>&1
s=$?; echo "kb decode exit $s"; tail -4 $O/kb_decode.log
[ $s -ne 0 ] && exit $s
timeout -k 10 300 python benchmarks/kernel_bench.py --only prefill > $O/kb_prefill.log 2>&1
s=$?; echo "kb prefill exit $s"; tail -4 $O/kb_prefill.log
[ $s -ne 0 ] && exit $s
timeout -k 10 300 python benchmarks/moe_bench.py > $O/moe.log 2>&1
s=$?; echo "moe exit $s"; cat $O/moe.log | tail -6
exit $s
