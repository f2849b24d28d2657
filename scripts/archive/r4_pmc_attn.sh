#!/usr/bin/env bash
# Round 4 counter passes with normalised / raw-request derivations (scripts/pmc_summary.py):
#   decode attention: HBM read bytes from TCC_EA0_RDREQ by request size vs the analytic KV bytes
#   prefill attention: MFMA utilisation (busy / 4 SIMDs x CU busy) and counter-implied FLOP/s vs analytic
#   skinny GEMM (o, M = 256): the same two
set -u
R="$(cd "$(dirname "$0")/.." && pwd)"
O="$R/gpurun_out/${1:-r4_pmc_attn}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
pass() {  # name, filter, command..., --, counters
  local name=$1 filt=$2; shift 2
  local cmd=()
  while [ "$1" != "--" ]; do cmd+=("$1"); shift; done; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$O/raw_$name" -o run -- \
      "${cmd[@]}" > "$O/$name.log" 2>&1
  local s=$?
  echo "$name exit $s"
  [ $s -eq 0 ] || return $s
  python3 "$R/scripts/pmc_summary.py" "$O/raw_$name" "$filt" > "$O/$name.txt" 2>&1
  rm -rf "$O/raw_$name"
}
KB="$R/benchmarks/kernel_bench.py"
pass decode_hbm decode_attn python3 "$KB" --only decode --iters 3 -- TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum || exit 1
pass prefill_mfma prefill_attn python3 "$KB" --only prefill --iters 3 -- SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit 1
pass skinny_hbm skinny python3 "$R/benchmarks/skinny_one.py" --shape o --m 256 --cfg 1 --split 4 --iters 40 -- TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum || exit 1
python3 "$KB" --only prefill --iters 5 > "$O/prefill_shapes.json" 2>&1
for f in "$O"/*.txt; do echo "== $f"; head -40 "$f"; done
