#!/usr/bin/env bash
# MoE grouped GEMM: numerics, then the Mixtral-layer micro-benchmark.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/${TAG:-r2_moe}"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_families_gpu.py -v -p no:cacheprovider -rf --timeout 120 --timeout-method thread -k "moe or mixtral" > $O/pytest_moe.log 2>&1
s=$?; echo "pytest exit $s"; grep -E "passed|failed|FAILED|Error" $O/pytest_moe.log | tail -8
[ $s -ne 0 ] && exit $s
timeout -k 10 300 python benchmarks/moe_bench.py > $O/moe.log 2>&1
s=$?; echo "moe exit $s"; grep tokens $O/moe.log
[ $s -ne 0 ] && exit $s
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw" -o run -- python3 "$R/benchmarks/moe_bench.py" --tokens ${MOE_TOKENS:-1536} > "$O/prof.log" 2>&1
s=$?; echo "prof exit $s"
python3 "$R/scripts/summarize_prof.py" "$O/raw" > "$O/kernels.txt" 2>&1
head -12 "$O/kernels.txt"
rm -rf "$O/raw"
exit $s
