#!/usr/bin/env bash
# FP8 KV cache on the headline workload (Llama-3-8B) and on KV-bound Gemma-7B
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
O="$R/gpurun_out/r2_kvfp8"; mkdir -p "$O"
for m in ${MODELS:-llama3-8b gemma-7b}; do
  timeout -k 10 420 python bench.py --model $m --steps ${STEPS:-3} --warmup 2 --kv-fp8 --out $O/bench_$m.json > $O/bench_$m.log 2>&1
  s=$?; echo "$m exit $s $(python -c "import json;d=json.load(open('$O/bench_$m.json'));print(d['value'],d['p50_latency_ms'],d['dtype'])" 2>/dev/null)"
  [ $s -ne 0 ] && exit $s
done
exit 0
