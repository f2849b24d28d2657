#!/usr/bin/env bash
# Sweep of the mixed-step prefill budget on the headline bench (default 2048).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r32"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
for m in 2048 1280 3072 2048; do
  timeout -k 10 600 python bench.py --steps 2 --warmup 1 --mixed-prefill-tokens $m --out "$O/bench_m$m.json" > "$O/bench_m$m.log" 2>&1 || { tail -20 "$O/bench_m$m.log"; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_m$m.json')); print($m, d['value'], d['p50_latency_ms'], d['p50_ttft_ms'])"
done
