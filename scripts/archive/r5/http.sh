#!/bin/bash
# Round 5: REST path, in-process and split topology (model server + chain server), per-token
# streaming (interval 1) and interval 8; each times 2,048 requests after 256 warm-up
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_http
mkdir -p $out
export NGA_HTTP_BENCH_LOG=$PWD/$out/server.log
for spec in "$@"; do
  topo=${spec%:*}; iv=${spec#*:}
  if [ "$topo" = "bench" ]; then
    timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench.json'));print('bench', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'])"
    continue
  fi
  [ -n "${PYSAMPLE:-}" ] && export NGA_PY_SAMPLE_OUT=$PWD/$out/pysample_${topo}_iv${iv}_{tag}.json
  timeout -k 10 600 python benchmarks/http_rag.py --topology $topo --stream-interval $iv --out $out/http_${topo}_iv$iv.json > $out/http_${topo}_iv$iv.log 2>&1 || { tail -30 $out/http_${topo}_iv$iv.log; tail -30 $out/server.log; exit 1; }
  python -c "import json;d=json.load(open('$out/http_${topo}_iv$iv.json'));print('$topo iv$iv', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'], d['sse_gap_ms'], d['server_p50_ms'])"
done
