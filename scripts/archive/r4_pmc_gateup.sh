#!/bin/bash
# Round 4: counter passes on the gate/up decode-shape GEMM (M = 256, cfg 13, SwiGLU epilogue):
# L2 -> CU read requests (x 128 B), their latency, HBM bytes, MFMA busy
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
O="$R/gpurun_out/r4_pmc_gateup"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1 args=$2; shift 2
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$O/raw_$name" -o run -- \
      python3 "$R/benchmarks/skinny_one.py" $args --iters 40 > "$O/$name.log" 2>&1
  local s=$?
  echo "$name exit $s"
  [ $s -eq 0 ] || return $s
  python3 "$R/scripts/pmc_summary.py" "$O/raw_$name" > "$O/$name.txt" 2>&1
  rm -rf "$O/raw_$name"
}
a="--shape gate_up --m 256 --cfg 13 --split 1"
pass gu_tcp "$a" TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TA_TCP_STATE_READ_sum || exit 1
pass gu_tccsz "$a" TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_TAG_STALL_sum || exit 1
pass gu_sq "$a" SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_TA_BUSY || exit 1
for f in "$O"/*.txt; do echo "== $f"; grep -A12 "skinny_gemm_kernel" "$f" | head -16; done
