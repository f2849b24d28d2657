#!/bin/bash
# Round 6: the driver's configuration on this tree, then the timed-window kernel trace
set -o pipefail
cd "$(dirname "$0")/../../.."
R=$PWD
out=gpurun_out/${1:-r6_final}
mkdir -p $out
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print('bench', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'], d['prefix_cache']['hit_share'], d['gpu_step_timing'])"
bash scripts/gpu_busy.sh ${1:-r6_final}_busy
