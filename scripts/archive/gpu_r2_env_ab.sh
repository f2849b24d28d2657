#!/usr/bin/env bash
# Headline A/B of a runtime environment setting (AB_ENV, e.g. HIP_FORCE_DEV_KERNARG=1),
# interleaved: default, setting, default, setting
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
O="$R/gpurun_out/env_ab"; mkdir -p "$O"
i=0
for v in base env base env; do
  i=$((i+1))
  if [ $v = env ]; then E="env $AB_ENV"; else E=""; fi
  timeout -k 10 300 $E python bench.py --steps 5 --warmup 2 --out $O/bench_${v}_r$i.json > $O/bench_${v}_r$i.log 2>&1
  s=$?; [ $s -ne 0 ] && { echo "bench $v exit $s"; tail -5 $O/bench_${v}_r$i.log; exit $s; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'QPS', d['value'], 'p50', d['p50_latency_ms'], 'ttft', d['p50_ttft_ms'])" $O/bench_${v}_r$i.json $v
done
