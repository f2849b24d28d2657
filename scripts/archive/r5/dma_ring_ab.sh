#!/bin/bash
# Round 5: whole-page LDS-DMA decode kernel (NGA_DECODE_DMA=1) vs its K / V^T refill ring (2),
# both with nt KV loads, decode step 256 x 1,400 interleaved x 2
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_dma_ring
mkdir -p $out
for r in 1 2; do
  for v in 1 2; do
    NGA_DECODE_DMA=$v timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 48 > $out/decode_${v}_$r.json 2> $out/decode_${v}_$r.err || { tail -5 $out/decode_${v}_$r.err; exit 1; }
    echo "decode dma $v round $r $(python3 -c "import json;d=json.load(open('$out/decode_${v}_$r.json'));print(d['replay_ms'], d['step_ms'])")"
  done
done
if [ "${1:-}" = "headline" ]; then
  for rv in "1 1" "2 1" "1 2" "2 2"; do
    set -- $rv; v=$1; r=$2
    NGA_DECODE_DMA=$v timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $out/bench_${v}_$r.json 2> $out/bench_${v}_$r.err || { tail -5 $out/bench_${v}_$r.err; exit 1; }
    echo "bench dma $v round $r $(python3 -c "import json;d=json.load(open('$out/bench_${v}_$r.json'));print(d['value'], d['p50_latency_ms'])")"
  done
fi
