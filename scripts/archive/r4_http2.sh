#!/bin/bash
# Round 4: REST-path RAG after the serving fixes (anyio pool, prompt queued from the worker thread,
# batched token deliveries + stream interval, batched context token counts); A/B over the
# GIL switch interval (APP_GIL_SWITCH_US) and the stream interval (NGA_STREAM_INTERVAL)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_http2; mkdir -p $O
for v in ${VARIANTS:-500:3 5000:3 200:3}; do
  sw=${v%%:*}; iv=${v##*:}; tag=sw${sw}_iv${iv}_qw${QW:-2}
  NGA_QUERY_BATCH_WAIT_MS=${QW:-2} APP_GIL_SWITCH_US=$sw NGA_STREAM_INTERVAL=$iv timeout -k 10 400 python -u benchmarks/http_rag.py --out $O/http_rag_$tag.json > $O/http_rag_$tag.log 2>&1 || { tail -30 $O/http_rag_$tag.log; tail -30 gpurun_out/http_rag_server.log; exit 1; }
  echo "$tag $(cat $O/http_rag_$tag.json)"
done
if [ -n "$WITH_BENCH" ]; then
  timeout -k 10 420 python -u bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'], d['host_s'], d['steps_prefill_decode_mixed'])"
fi
