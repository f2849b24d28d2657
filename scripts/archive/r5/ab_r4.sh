#!/bin/bash
# Round 5: same-box A/B of the headline and the 256 x 1,400 decode step, round-4 tree (ab_r4/,
# a git worktree of c3260e5 built in place) vs this tree, interleaved
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_ab_r4
mkdir -p $out
for i in 1 2; do
  for t in r4 r5; do
    d=.; [ $t = r4 ] && d=ab_r4
    (cd $d && timeout -k 10 400 python bench.py --steps 10 --warmup 3) > $out/bench_${t}_$i.json 2> $out/bench_${t}_$i.err || { tail -20 $out/bench_${t}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_${t}_$i.json'));print('$t', $i, d['value'], d['p50_latency_ms'], d['p50_ttft_ms'])"
  done
done
for t in r4 r5; do
  d=.; [ $t = r4 ] && d=ab_r4
  (cd $d && timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16) > $out/decode_$t.json 2> $out/decode_$t.err || { tail -20 $out/decode_$t.err; exit 1; }
  echo $t $(tail -1 $out/decode_$t.json)
done
