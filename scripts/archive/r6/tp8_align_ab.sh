#!/bin/bash
# Round 6: the alignment rule on the TP = 8 agent rehearsal (8 ranks on one GPU), new vs old
# (NGA_ALIGN_OLD was a temporary switch in scheduler.cpp, removed again after this A/B)
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/r6_tp8_align
mkdir -p $out
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=2
for i in 1 2; do
  for old in 0 1; do
    NGA_ALIGN_OLD=$old timeout -k 10 420 python bench.py --gpus 8 --tp 8 --workload agent --model llama70b-small --allow-shared-devices --steps 4 --warmup 1 --concurrency 16 --max-tokens 128 --kv-cache-fraction 0.04 --out $out/bench_old${old}_$i.json > $out/bench_old${old}_$i.log 2>&1 || { echo "rc=$? old=$old"; tail -20 $out/bench_old${old}_$i.log; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_old${old}_$i.json'));print('old=$old', d['value'], d['p50_latency_ms'])"
  done
done
