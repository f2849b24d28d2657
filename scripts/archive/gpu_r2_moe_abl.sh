#!/usr/bin/env bash
# MoE grouped GEMM ablation: normal, no-DMA, no-MFMA builds.
# needs the diagnostic build: NGA_DIAG_BUILD=1 python -c 'from nv_genai_amd._build import build_kernels; build_kernels(force=True)'
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r2_moe_abl"; mkdir -p "$O"
for a in ${ABLS:-0 1 2}; do
  NGA_MOE_ABLATE=$a timeout -k 10 120 python benchmarks/moe_bench.py --gemm-only --tokens ${TOKS:-256,1536,4096} > $O/abl_$a.log 2>&1
  s=$?; echo "ablate $a exit $s"; grep tokens $O/abl_$a.log
  [ $s -ne 0 ] && exit $s
done
exit 0
