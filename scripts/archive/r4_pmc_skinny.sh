#!/bin/bash
# Round 4: counter passes on the skinny GEMM (o projection, M = 256, cfg 1, split 4) and the
# library GEMM of the same shape; new GPU tests; the REST-path headline (http_rag).
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
O="$R/gpurun_out/r4_pmc"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
pass() {  # name, args for skinny_one, counters...
  local name=$1 args=$2; shift 2
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$O/raw_$name" -o run -- \
      python3 "$R/benchmarks/skinny_one.py" $args --iters 60 > "$O/$name.log" 2>&1
  local s=$?
  echo "$name exit $s"
  [ $s -eq 0 ] || return $s
  python3 "$R/scripts/pmc_summary.py" "$O/raw_$name" > "$O/$name.txt" 2>&1
  rm -rf "$O/raw_$name"
}
for v in "sk:--shape o --m 256 --cfg 1 --split 4" "lib:--shape o --m 256 --lib"; do
  n=${v%%:*}; a=${v#*:}
  pass ${n}_tcc "$a" TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum || exit 1
  pass ${n}_tccsz "$a" TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_TAG_STALL_sum || exit 1
  pass ${n}_tcp "$a" TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TA_TCP_STATE_READ_sum || exit 1
  pass ${n}_sq "$a" SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_TA_BUSY || exit 1
  pass ${n}_ta "$a" TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum || exit 1
done
for f in "$O"/*.txt; do echo "== $f"; cat "$f"; done
cd "$R"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "gqa_4096" tests/test_search_gpu.py::test_ivf_scan_splits_past_item_limit > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
tail -4 "$O/tests.txt"
