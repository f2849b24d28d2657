#!/usr/bin/env bash
# Headline bench across mixed-step prefill budgets (CFGS: "tokens:min_tokens" pairs)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
O="$R/gpurun_out/r2_mixed_sweep"; mkdir -p "$O"
i=0
for c in ${CFGS:-2048:0 3072:0 4096:0 2048:1024}; do
  t=${c%%:*}; m=${c##*:}; i=$((i+1))
  timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 2 --mixed-prefill-tokens $t --mixed-min-tokens $m \
    --out $O/bench_${t}_${m}_r$i.json > $O/bench_${t}_${m}_r$i.log 2>&1
  s=$?; [ $s -ne 0 ] && { echo "bench $c exit $s"; tail -5 $O/bench_${t}_${m}_r$i.log; exit $s; }
  python - "$O/bench_${t}_${m}_r$i.json" "$c" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "QPS", d["value"], "p50", d["p50_latency_ms"], "ttft", d["p50_ttft_ms"], "steps", d["steps_prefill_decode_mixed"])
PY
done
