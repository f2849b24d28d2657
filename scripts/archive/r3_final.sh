#!/bin/bash
# Round-3 checkpoint: whole GPU suite + smoke + headline kernel profile (r3_full_gpu.sh), then
# the headline bench at the driver's configuration.
set -o pipefail
N=${1:-r3_final2}
bash scripts/r3_full_gpu.sh $N || exit 1
cat gpurun_out/${N}_prof/attn_overlap.json 2>/dev/null
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/$N/bench.json 2> gpurun_out/$N/bench.err || { tail -20 gpurun_out/$N/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/$N/bench.json'));print(d['value'],d['p50_latency_ms'],d['p50_ttft_ms'],d['host_s'],d['submit_host_ms'])"
