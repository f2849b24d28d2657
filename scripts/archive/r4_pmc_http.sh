#!/bin/bash
# Round 4: counter passes (attention + skinny) and the REST-path headline on the current tree
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/r4_pmc_attn.sh r4_pmc_attn || exit 1
O=gpurun_out/r4_http; mkdir -p $O
timeout -k 10 700 python -u benchmarks/http_rag.py --out $O/http_rag.json > $O/http_rag.log 2>&1 || { tail -30 $O/http_rag.log; tail -30 gpurun_out/http_rag_server.log; exit 1; }
cat $O/http_rag.json
