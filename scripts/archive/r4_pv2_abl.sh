#!/bin/bash
# Round 4: prefill v2 ablations at the serving shapes (diagnostic build; timings only):
# 0 = shipped, 8 = V DMA a whole iteration ahead (racy), 16 = no vmcnt wait before the barrier
O=gpurun_out/r4_pv2_abl; mkdir -p $O
for a in ${ABLS:-0 8 16 1}; do
  NGA_PV2_ABLATE=$a timeout -k 10 120 python -u benchmarks/kernel_bench.py --only prefill > $O/abl_$a.json 2> $O/abl_$a.err
  s=$?; [ $s -ne 0 ] && { tail -5 $O/abl_$a.err; exit $s; }
  python3 -c "
import json; d=json.load(open('$O/abl_$a.json'))
print('abl $a', {k: v['mfma32']['us'] for k, v in d.items() if k.startswith('prefill')})"
done
exit 0
