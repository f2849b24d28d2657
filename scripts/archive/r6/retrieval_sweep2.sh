#!/bin/bash
# Round 6: retrieval batching (--retrieval-batch queries per embedding + search launch,
# --retrieval-delay-ms max wait for the batch to fill), interleaved on one box: headline (8 steps)
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_retrieval2}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for i in 1 2; do
  for cfg in 8:50 8:100 16:50 16:100; do
    b=${cfg%%:*}; dl=${cfg##*:}
    timeout -k 10 400 python bench.py --steps 8 --warmup 2 --retrieval-batch $b --retrieval-delay-ms $dl > $out/bench_b${b}_d${dl}_$i.json 2> $out/bench_b${b}_d${dl}_$i.err || { tail -20 $out/bench_b${b}_d${dl}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_b${b}_d${dl}_$i.json'));print('batch=$b delay=$dl', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'], d['host_work_ms']['submit'][0])"
  done
done
