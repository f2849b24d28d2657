#!/bin/bash
# Round 6: retrieval batching delay (--retrieval-delay-ms, the max time a query waits for its
# embedding + search batch to fill), interleaved on one box: headline (8 steps)
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_retrieval}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for i in 1 2; do
  for dl in 50 20 8; do
    timeout -k 10 400 python bench.py --steps 8 --warmup 2 --retrieval-delay-ms $dl > $out/bench_d${dl}_$i.json 2> $out/bench_d${dl}_$i.err || { tail -20 $out/bench_d${dl}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_d${dl}_$i.json'));print('delay=$dl', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'], d['host_work_ms']['submit'][0], d['submit_host_ms'])"
  done
done
