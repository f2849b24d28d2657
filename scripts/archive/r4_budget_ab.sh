#!/bin/bash
# Round 4: headline vs the mixed-step prefill budget (interleaved), with the decode-shape kernels in
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_budget_ab; mkdir -p $O
i=0
for v in ${BUDGETS:-4096 5120 3072 4096 5120}; do
  i=$((i+1))
  timeout -k 10 420 python -u bench.py --steps 10 --warmup 3 --mixed-prefill-tokens $v > $O/bench_${i}_$v.json 2> $O/bench_${i}_$v.err || { tail -20 $O/bench_${i}_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_${i}_$v.json'));print('budget $v', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'])"
done
