#!/bin/bash
# Round 6: the scheduler's token alignment A/B, interleaved on one box: headline (8 steps) with
# the step timeline of each run. NGA_ALIGN_OLD was a temporary switch in scheduler.cpp (0 = no
# cut that leaves a prompt tail shorter than one alignment unit, shipped; 1 = the old rule; 2 =
# tails finished in one padded step); the shipped tree has rule 0 only.
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_align}
rules=${2:-"0 1"}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for i in 1 2; do
  for old in $rules; do
    NGA_ALIGN_OLD=$old timeout -k 10 400 python bench.py --steps 8 --warmup 2 --timeline-out $out/tl_old${old}_$i.json > $out/bench_old${old}_$i.json 2> $out/bench_old${old}_$i.err || { tail -20 $out/bench_old${old}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_old${old}_$i.json'));print('rule=$old', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'], d['gpu_step_timing']['steps'], d['step_graphs']['launches_by_token_bucket'])"
    python scripts/steps_probe.py $out/tl_old${old}_$i.json > $out/steps_old${old}_$i.json
  done
done
