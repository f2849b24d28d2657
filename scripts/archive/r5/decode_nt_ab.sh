#!/bin/bash
# Round 5: decode_nt (nt KV loads in the register decode kernel, the one fp8 KV pages use) A/B:
# the bf16 decode step forced onto the register kernel (NGA_DECODE_DMA=0) interleaved 0/1 x 2,
# then the fp8 headline (bench.py --fp8 --kv-fp8, 8 steps / 2 warm-up) interleaved 0/1 x 2
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_decode_nt
mkdir -p $out
for r in 1 2; do
  for v in 0 1; do
    NGA_DECODE_DMA=0 NGA_DECODE_NT=$v timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 48 > $out/decode_reg_${v}_$r.json 2> $out/decode_reg_${v}_$r.err || { tail -5 $out/decode_reg_${v}_$r.err; exit 1; }
    echo "decode (register kernel) nt $v round $r $(python3 -c "import json;d=json.load(open('$out/decode_reg_${v}_$r.json'));print(d['replay_ms'], d['step_ms'])")"
  done
done
for rv in "0 1" "1 1" "0 2" "1 2"; do
  set -- $rv; v=$1; r=$2
  NGA_DECODE_NT=$v timeout -k 10 300 python bench.py --steps 8 --warmup 2 --fp8 --kv-fp8 > $out/bench_fp8_${v}_$r.json 2> $out/bench_fp8_${v}_$r.err || { tail -5 $out/bench_fp8_${v}_$r.err; exit 1; }
  echo "bench fp8 nt $v round $r $(python3 -c "import json;d=json.load(open('$out/bench_fp8_${v}_$r.json'));print(d['value'], d['p50_latency_ms'])")"
done
