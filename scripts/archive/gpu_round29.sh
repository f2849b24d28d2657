#!/usr/bin/env bash
# Agent config with Llama-3-70B in FP8 W8A8 (70 GB of weights) on one MI355X.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r29"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python benchmarks/agent_tp.py --model llama3-70b --fp8 --index-size 10000000 --queries 64 \
    --concurrency 32 --out "$O/agent_70b_fp8.json" > "$O/agent_70b_fp8.log" 2>&1 || { tail -20 "$O/agent_70b_fp8.log"; exit 1; }
cat "$O/agent_70b_fp8.json"
