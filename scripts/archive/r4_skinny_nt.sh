#!/bin/bash
# Round 4: skinny GEMM with non-temporal weight DMA (NGA_SKINNY_WNT=1) vs default, M = 64 / 128 / 256
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_skinny_nt; mkdir -p $O
for wnt in 0 1; do
  NGA_SKINNY_WNT=$wnt timeout -k 10 300 python -u benchmarks/skinny_gemm.py --ms 64,128,256 --shapes o,qkv,down,gate_up --cfgs 0,1,2,3,10,12,13,16 > $O/sweep_wnt$wnt.jsonl 2>&1 || { tail -20 $O/sweep_wnt$wnt.jsonl; exit 1; }
  echo "== wnt $wnt"; grep '"lib_us"' $O/sweep_wnt$wnt.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); b=r['best_gemm']; print(r['shape'], r['M'], 'lib', r['lib_us'], 'best', b['cfg'], b['split'], b['gemm_us'], b['total_us'])"
done
