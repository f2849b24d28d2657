#!/bin/bash
# Round 5: the other BASELINE.json configs on the final tree: multi-turn RAG (64 sessions) and
# the query-decomposition agent with Llama-3-8B over a 10M-vector index (1 GPU)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5_configs; mkdir -p $O
timeout -k 10 500 python -u benchmarks/multi_turn.py --out $O/multi_turn.json > $O/multi_turn.log 2>&1 || { tail -20 $O/multi_turn.log; exit 1; }
echo "multi-turn: $(python3 -c "import json;d=json.load(open('$O/multi_turn.json'));print(d['value'], d.get('p50_latency_ms'))")"
timeout -k 10 500 python -u benchmarks/agent_tp.py --model llama3-8b --index-size 10000000 --out $O/agent8b.json > $O/agent8b.log 2>&1 || { tail -20 $O/agent8b.log; exit 1; }
echo "agent 8b: $(python3 -c "import json;d=json.load(open('$O/agent8b.json'));print(d['value'], d.get('p50_latency_ms'))")"
if [ "${1:-}" = "70b" ]; then
  timeout -k 10 700 python -u benchmarks/agent_tp.py --model llama3-70b --index-size 10000000 --out $O/agent70b.json > $O/agent70b.log 2>&1 || { tail -20 $O/agent70b.log; exit 1; }
  echo "agent 70b: $(python3 -c "import json;d=json.load(open('$O/agent70b.json'));print(d['value'], d.get('p50_latency_ms'))")"
fi
