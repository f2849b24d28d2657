#!/bin/bash
# v2 prefill attention ablations (NGA_PV2_ABLATE; timings only, results are wrong)
# needs the diagnostic build: NGA_DIAG_BUILD=1 python -c 'from nv_genai_amd._build import build_kernels; build_kernels(force=True)'
O=gpurun_out/r2_pv2; mkdir -p $O
for a in ${ABLS:-0 1 2 3 4}; do
  NGA_PV2_ABLATE=$a timeout -k 10 120 python -u benchmarks/kernel_bench.py --only prefill > $O/abl_$a.json 2> $O/abl_$a.err
  s=$?; echo "abl $a: $(cat $O/abl_$a.json)"; [ $s -ne 0 ] && exit $s
done
exit 0
