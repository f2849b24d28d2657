#!/bin/bash
# Round 4: headline bench at the driver's configuration (20 steps, 5 warm-up), then the kernel profile
set -o pipefail
N=${1:-r4_final}
mkdir -p gpurun_out/$N
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/$N/bench.json 2> gpurun_out/$N/bench.err || { tail -20 gpurun_out/$N/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/$N/bench.json'));print(d['value'],d['p50_latency_ms'],d['p50_ttft_ms'],d['host_s'],d.get('gpu_step_timing'))"
bash scripts/r3_prof.sh ${N}_prof && head -30 gpurun_out/${N}_prof/kernels.txt
