#!/usr/bin/env bash
# Multi-turn RAG config (BASELINE configs[2]) on one MI355X.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r24"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python benchmarks/multi_turn.py --sessions 64 --turns 4 --out "$O/multi_turn_s64.json" \
    > "$O/multi_turn_s64.log" 2>&1 || { tail -20 "$O/multi_turn_s64.log"; exit 1; }
cat "$O/multi_turn_s64.json"
timeout -k 10 600 python benchmarks/multi_turn.py --sessions 128 --turns 4 --out "$O/multi_turn_s128.json" \
    > "$O/multi_turn_s128.log" 2>&1 || { tail -20 "$O/multi_turn_s128.log"; exit 1; }
cat "$O/multi_turn_s128.json"
