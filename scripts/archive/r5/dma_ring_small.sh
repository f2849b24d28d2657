#!/bin/bash
# Round 5: ring (2) vs whole-page (1) LDS-DMA decode kernel at small decode batches
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_dma_ring_small
mkdir -p $out
for b in 16 64; do
  for r in 1 2; do
    for v in 1 2; do
      NGA_DECODE_DMA=$v timeout -k 10 200 python benchmarks/decode_step.py --batch $b --ctx 1400 --steps 48 > $out/decode_b${b}_${v}_$r.json 2> $out/decode_b${b}_${v}_$r.err || { tail -5 $out/decode_b${b}_${v}_$r.err; exit 1; }
      echo "batch $b dma $v round $r $(python3 -c "import json;d=json.load(open('$out/decode_b${b}_${v}_$r.json'));print(d['replay_ms'], d['step_ms'])")"
    done
  done
done
