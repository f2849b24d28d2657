#!/bin/bash
# Round 6: the TP = 8 agent (BASELINE.json configs[3]) rehearsed with 8 ranks on the one GPU:
# llama70b-small (70B head layout), 10M-vector index sharded 8 ways; the new search path
# (queries in the step-channel command + one IPC all-gather) against the round-5 one
# (broadcast + process-group gathers), then bench.py's record of the same job
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_tp8_agent}
mkdir -p $out
export PYTHONUNBUFFERED=1 GPU_MAX_HW_QUEUES=2
A="--model llama70b-small --index-size 10000000 --queries 64 --warmup 16 --concurrency 16 --answer-tokens 128 --kv-cache-fraction 0.04"
for v in new legacy; do
  extra=""; [ $v = legacy ] && extra="--search-legacy"
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29611 \
    benchmarks/agent_tp.py $A $extra --out $out/agent_$v.json > $out/agent_$v.log 2>&1 || { echo "rc=$? $v"; tail -20 $out/agent_$v.log; exit 1; }
  python -c "import json;d=json.load(open('$out/agent_$v.json'));print('$v', d['value'], d['p50_latency_ms'], d['search'])"
done
timeout -k 10 420 python bench.py --gpus 8 --tp 8 --workload agent --model llama70b-small --allow-shared-devices \
  --steps 4 --warmup 1 --concurrency 16 --max-tokens 128 --kv-cache-fraction 0.04 --out $out/bench_agent_tp8.json > $out/bench.log 2>&1 || { echo "rc=$? bench"; tail -20 $out/bench.log; exit 1; }
python -c "import json;d=json.load(open('$out/bench_agent_tp8.json'));print('bench', d['value'], d['search'], [r.get('custom_all_reduce') for r in d['devices']['ranks']][:2], [(r.get('cpu_affinity'), r.get('physical_cores')) for r in d['devices']['ranks']][:3])"
