#!/usr/bin/env bash
# Prefill accumulation sweep for the closed-loop bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "mm0:--mixed-min-tokens 0" "mm2300:--mixed-min-tokens 2300 --mixed-prefill-tokens 4096" "mm3500:--mixed-min-tokens 3500 --mixed-prefill-tokens 4096 --mixed-max-wait 6" "mm3500_c288:--mixed-min-tokens 3500 --mixed-prefill-tokens 4096 --mixed-max-wait 6 --concurrency 288"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 600 python bench.py --steps 2 --warmup 1 $args --out gpurun_out/bench_$name.json > gpurun_out/bench_$name.log 2>&1 || exit $?
  python - "$name" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/bench_{sys.argv[1]}.json"))
print(sys.argv[1], d["value"], d["p50_latency_ms"], d["p50_ttft_ms"], d["steps_prefill_decode_mixed"])
PY
done
