#!/bin/bash
# Round 5: decode-shape GEMM with weights rotating past the MALL (cold, as in a decode step)
# vs one cache-warm copy: how much of its time is the latency of HBM-sourced weight tiles?
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_hotcold
mkdir -p $out
: > $out/hotcold.jsonl
for rot in 640 0; do
  for s in o down gate_up; do
    timeout -k 10 150 python -u benchmarks/skinny_gemm.py --shapes $s --ms 256 --cfgs 1,12,13,16 --iters 30 --rot-mb $rot > $out/tmp.jsonl 2>&1 || { tail -20 $out/tmp.jsonl; exit 1; }
    grep '"lib_us"' $out/tmp.jsonl | sed "s/^{/{\"rot_mb\": $rot, /" >> $out/hotcold.jsonl
  done
done
cat $out/hotcold.jsonl | cut -c1-400
