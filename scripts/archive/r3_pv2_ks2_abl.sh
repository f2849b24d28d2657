#!/bin/bash
# Split-key (KS = 2) prefill ablations at few-prompt shapes (diagnostic build: NGA_DIAG_BUILD=1;
# NGA_PV2_ABLATE 1 = no DMA in the loop, 4 = no DMA and no barrier; timings only).
O=gpurun_out/r3_pv2_ks2; mkdir -p $O
for a in ${ABLS:-0 1 4}; do
  NGA_PV2_ABLATE=$a timeout -k 10 200 python -u benchmarks/kernel_bench.py --only prefill > $O/abl_$a.json 2> $O/abl_$a.err
  s=$?; echo "abl $a: $(python -c "import json;d=json.load(open('$O/abl_$a.json'));print({k:v['mfma32_ks2'] for k,v in d.items()})")"; [ $s -ne 0 ] && exit $s
done
exit 0
