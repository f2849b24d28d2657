#!/usr/bin/env bash
# End-to-end RAG through the chain-server REST API on one MI355X (256 concurrent SSE clients).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r31"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
NGA_HTTP_BENCH_LOG="$O/server.log" timeout -k 10 900 python benchmarks/http_rag.py --concurrency 256 --requests 512 \
    --warmup 256 --out "$O/http_rag.json" > "$O/http_rag.log" 2>&1 || { tail -20 "$O/http_rag.log"; tail -20 "$O/server.log"; exit 1; }
cat "$O/http_rag.json"
