#!/usr/bin/env bash
# Streaming-ingest throughput (MiniLM as in the reference's Triton pipeline, and arctic-embed-l).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r34"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
for m in all-minilm-l6-v2 arctic-embed-l; do
  timeout -k 10 600 python benchmarks/ingest_rate.py --docs 4000 --embed-model $m --threads 8 --out "$O/ingest_$m.json" > "$O/ingest_$m.log" 2>&1 || { tail -20 "$O/ingest_$m.log"; exit 1; }
  cat "$O/ingest_$m.json"
done
