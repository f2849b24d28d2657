#!/bin/bash
# Round 5: rope_vnt (non-temporal V^T page stores: 1 all, 2 decode rows only) A/B where it
# matters: the decode step interleaved 0/1/2 x 2, then the headline (8 steps / 2 warm-up)
# interleaved 0/2 x 2 and 1 once
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_rope_vnt_ab
mkdir -p $out
for r in 1 2; do
  for v in 0 1 2; do
    NGA_ROPE_VNT=$v timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 48 > $out/decode_${v}_$r.json 2> $out/decode_${v}_$r.err || { tail -5 $out/decode_${v}_$r.err; exit 1; }
    echo "decode vnt $v round $r $(python3 -c "import json;d=json.load(open('$out/decode_${v}_$r.json'));print(d['replay_ms'], d['step_ms'])")"
  done
done
for rv in "0 1" "2 1" "0 2" "2 2" "1 1"; do
  set -- $rv; v=$1; r=$2
  NGA_ROPE_VNT=$v timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $out/bench_${v}_$r.json 2> $out/bench_${v}_$r.err || { tail -5 $out/bench_${v}_$r.err; exit 1; }
  echo "bench vnt $v round $r $(python3 -c "import json;d=json.load(open('$out/bench_${v}_$r.json'));print(d['value'], d['p50_latency_ms'])")"
done
