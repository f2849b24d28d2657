#!/usr/bin/env bash
# Round-3 counter passes (each its own rocprofv3 run, kernel trace only beside --pmc):
#   decode attention  FETCH_SIZE (HBM bytes) + SQ stall mix, kernel_bench --only decode
#   prefill attention SQ MFMA-busy / LDS bank conflicts / wait mix, kernel_bench --only prefill
# Summaries joined per dispatch by scripts/pmc_summary.py; raw CSVs are dropped.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r3_pmc}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
pass() {  # name, kernel_bench --only, kernel filter, counters...
  local name=$1 only=$2 filt=$3; shift 3
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$O/raw_$name" -o run -- \
      python3 "$R/benchmarks/kernel_bench.py" --only "$only" --iters 3 > "$O/$name.log" 2>&1
  local s=$?
  echo "$name exit $s"
  [ $s -eq 0 ] || return $s
  python3 "$R/scripts/pmc_summary.py" "$O/raw_$name" "$filt" > "$O/$name.txt" 2>&1
  rm -rf "$O/raw_$name"
}
pass decode_fetch decode decode_attn FETCH_SIZE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM || exit 1
pass prefill_sq prefill prefill_attn SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS || exit 1
