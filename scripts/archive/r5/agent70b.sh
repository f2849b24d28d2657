#!/bin/bash
# Round 5: the query-decomposition agent with Llama-3-70B at TP=1 (141 GB of bf16 weights on
# one MI355X) over a 10M-vector index, final tree. The benchmark prints only at the end, so a
# heartbeat line goes to stdout every minute while it runs.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5_configs; mkdir -p $O
timeout -k 10 900 python -u benchmarks/agent_tp.py --model llama3-70b --index-size 10000000 --out $O/agent70b.json > $O/agent70b.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; echo "agent70b running $(date +%T)"; done
wait $pid || { tail -20 $O/agent70b.log; exit 1; }
echo "agent 70b: $(python3 -c "import json;d=json.load(open('$O/agent70b.json'));print(d['value'], d.get('p50_latency_ms'), d.get('llm_calls_per_s'))")"
