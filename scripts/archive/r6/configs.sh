#!/bin/bash
# Round 6: the other BASELINE.json configs on this tree. Mode "small" (default): multi-turn RAG,
# the agent with Llama-3-8B over a 10M-vector index, the REST path in the reference's split
# topology. Mode "70b": the agent with Llama-3-70B at TP = 1.
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/${1:-r6_configs}; mkdir -p $O
export PYTHONUNBUFFERED=1
val() { python3 -c "import json;d=json.load(open('$1'));print(d['value'], d.get('p50_latency_ms'), d.get('p50_ttft_ms', ''))"; }
if [ "${2:-small}" = "70b" ]; then
  timeout -k 10 900 python -u benchmarks/agent_tp.py --model llama3-70b --index-size 10000000 --out $O/agent70b.json > $O/agent70b.log 2>&1 || { tail -20 $O/agent70b.log; exit 1; }
  echo "agent 70b: $(val $O/agent70b.json)"
  exit 0
fi
timeout -k 10 500 python -u benchmarks/multi_turn.py --out $O/multi_turn.json > $O/multi_turn.log 2>&1 || { tail -20 $O/multi_turn.log; exit 1; }
echo "multi-turn: $(val $O/multi_turn.json)"
timeout -k 10 500 python -u benchmarks/agent_tp.py --model llama3-8b --index-size 10000000 --out $O/agent8b.json > $O/agent8b.log 2>&1 || { tail -20 $O/agent8b.log; exit 1; }
echo "agent 8b: $(val $O/agent8b.json)"
export NGA_HTTP_BENCH_LOG=$PWD/$O/server.log
timeout -k 10 600 python benchmarks/http_rag.py --topology split --stream-interval 1 --out $O/http_split_iv1.json > $O/http_split.log 2>&1 || { tail -30 $O/http_split.log; tail -30 $O/server.log; exit 1; }
echo "http split iv1: $(val $O/http_split_iv1.json)"
