#!/bin/bash
# Round 4: MFMA utilisation of the tuned library GEMMs of a full mixed step (M = 4,352 rows)
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
O="$R/gpurun_out/r4_pmc_libgemm"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for shp in gate_up down qkv o; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE --output-format csv -d "$O/raw_$shp" -o run -- \
      python3 "$R/benchmarks/skinny_one.py" --shape $shp --m 4352 --lib --tuned --iters 20 > "$O/$shp.log" 2>&1 || { echo "$shp failed"; exit 1; }
  python3 "$R/scripts/pmc_summary.py" "$O/raw_$shp" > "$O/$shp.txt" 2>&1
  rm -rf "$O/raw_$shp"
  echo "== $shp"; grep -B1 -A6 "Cijk" "$O/$shp.txt" | grep -E "Cijk|utilisation|implied|mean_us" | head -6
done
