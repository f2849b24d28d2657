#!/bin/bash
# Round 5: TP=2 rehearsal on one GPU (pipelined, graphed), headline with and without the prefix cache
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/${1:-r5_bench}
mkdir -p $out
timeout -k 10 420 python bench.py --gpus 2 --tp 2 --allow-shared-devices --steps 3 --warmup 1 > $out/tp2.json 2> $out/tp2.err || { tail -30 $out/tp2.err; exit 1; }
python -c "import json;d=json.load(open('$out/tp2.json'));print('tp2', d['value'], d['unpipelined_steps'], d['step_graphs']['timed_graph_steps'], d['devices']['ranks'][0].get('custom_all_reduce'))"
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('default', d['value'],d['p50_latency_ms'],d['p50_ttft_ms'],d['prefix_cache'])"
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-prefix-cache > $out/bench_nopc.json 2> $out/bench_nopc.err || { tail -20 $out/bench_nopc.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench_nopc.json'));print('no-prefix-cache', d['value'],d['p50_latency_ms'],d['p50_ttft_ms'],d['prefix_cache'])"
