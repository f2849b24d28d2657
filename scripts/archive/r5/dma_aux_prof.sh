#!/bin/bash
# Round 5: where the decode step's 4 % goes with the decode attention's KV DMA on the default
# cache policy (NGA_DECODE_DMA_AUX=0) vs nt (2): per-kernel times of the 256 x 1,400 decode step
set -o pipefail
cd "$(dirname "$0")/../.."
R=$PWD
out=gpurun_out/r5_dma_aux_prof
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for v in 2 0; do
  export NGA_DECODE_DMA_AUX=$v
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/raw_$v -o run -- python3 $R/benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 > $R/$out/prof_$v.log 2>&1 || { tail -20 $R/$out/prof_$v.log; exit 1; }
  python3 $R/scripts/summarize_prof.py $R/$out/raw_$v > $R/$out/kernels_aux$v.txt 2>&1
  rm -rf $R/$out/raw_$v
  head -16 $R/$out/kernels_aux$v.txt
done
