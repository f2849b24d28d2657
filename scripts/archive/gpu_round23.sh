#!/usr/bin/env bash
# Query-decomposition agent config (BASELINE configs[3]) on one MI355X: 10M-vector index,
# Llama-3-8B then Llama-3-70B (bf16, 141 GB of weights fit in 288 GB HBM) at TP=1.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r23"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python benchmarks/agent_tp.py --model llama3-8b --index-size 10000000 --queries 64 \
    --concurrency 32 --out "$O/agent_8b.json" > "$O/agent_8b.log" 2>&1 || { tail -20 "$O/agent_8b.log"; exit 1; }
cat "$O/agent_8b.json"
timeout -k 10 900 python benchmarks/agent_tp.py --model llama3-70b --index-size 10000000 --queries 64 \
    --concurrency 32 --out "$O/agent_70b.json" > "$O/agent_70b.log" 2>&1 || { tail -20 "$O/agent_70b.log"; exit 1; }
cat "$O/agent_70b.json"
