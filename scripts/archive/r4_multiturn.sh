#!/bin/bash
# Round 4: multi-turn RAG (64 sessions) and the 8B agent with the decode-shape kernels off / on
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_multiturn; mkdir -p $O
for v in 0 1; do
  NGA_SKINNY=$v timeout -k 10 500 python -u benchmarks/multi_turn.py --out $O/mt_sk$v.json > $O/mt_sk$v.log 2>&1 || { tail -20 $O/mt_sk$v.log; exit 1; }
  echo "multi-turn skinny $v: $(python3 -c "import json;d=json.load(open('$O/mt_sk$v.json'));print(d['value'], d.get('p50_latency_ms'))")"
  NGA_SKINNY=$v timeout -k 10 500 python -u benchmarks/agent_tp.py --model llama3-8b --index-size 10000000 --out $O/agent8b_sk$v.json > $O/agent8b_sk$v.log 2>&1 || { tail -20 $O/agent8b_sk$v.log; exit 1; }
  echo "agent 8b skinny $v: $(python3 -c "import json;d=json.load(open('$O/agent8b_sk$v.json'));print(d['value'], d.get('p50_latency_ms'))")"
done
