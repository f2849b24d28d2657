#!/usr/bin/env bash
# A/B of the mixed-step attention configuration on the headline bench (VARIANTS: names below)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
O="$R/gpurun_out/r2_attn_ab"; mkdir -p "$O"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 2 --out $O/$n.json > $O/$n.log 2>&1
  local s=$?; echo "$n exit $s $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['p50_latency_ms'])" 2>/dev/null)"
  return $s
}
for v in ${VARIANTS:-auto v1 v2}; do
  case $v in
    auto) run auto NGA_CONCURRENT_ATTN=1 || exit 1 ;;
    v1) run v1 NGA_PREFILL_V1=1 || exit 1 ;;
    serial) run serial NGA_CONCURRENT_ATTN=0 || exit 1 ;;
  esac
done
