#!/usr/bin/env bash
# Closed-loop bench with non-blocking retrieval: default, bigger prefill share, more clients.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "c256_m2048:--concurrency 256 --mixed-prefill-tokens 2048" "c256_m4096:--concurrency 256 --mixed-prefill-tokens 4096" "c320_m2048:--concurrency 320 --mixed-prefill-tokens 2048"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 600 python bench.py --steps 2 --warmup 1 $args --out gpurun_out/bench_$name.json > gpurun_out/bench_$name.log 2>&1 || exit $?
  echo "$name"; tail -1 gpurun_out/bench_$name.log
done
