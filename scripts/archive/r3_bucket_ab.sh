#!/usr/bin/env bash
# Headline A/B of the step-graph token bucket (256 / 128 / 64 tokens), interleaved on one box,
# with the GEMM table tuned at 64-token steps.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
O="$R/gpurun_out/${1:-r3_bucket}"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
i=0
for t in ${STEPS_LIST:-256 64 128 256 64 128}; do
  i=$((i+1))
  timeout -k 10 420 python bench.py --steps 5 --warmup 2 --graph-token-step $t > "$O/bench_${t}_r$i.json" 2> "$O/bench_${t}_r$i.err"
  s=$?; [ $s -ne 0 ] && { echo "bench $t exit $s"; tail -5 "$O/bench_${t}_r$i.err"; exit $s; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'QPS', d['value'], 'p50', d['p50_latency_ms'], 'graphs', d['step_graphs'])" "$O/bench_${t}_r$i.json" $t
done
