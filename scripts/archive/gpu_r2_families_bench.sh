#!/usr/bin/env bash
# Headline RAG workload on the other decoder families + the VLM describe rate (1 GPU).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r2_fambench"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
for m in ${MODELS:-mistral-7b gemma-7b starcoder2-15b}; do
  timeout -k 10 420 python bench.py --model $m --steps 2 --warmup 1 --out $O/bench_$m.json > $O/bench_$m.log 2>&1
  s=$?; echo "$m exit $s"; python3 -c "import json;d=json.load(open('$O/bench_$m.json'));print(d['config']['model'],d['value'],d['p50_latency_ms'],d['output_tokens_per_s'])"
  [ $s -ne 0 ] && exit $s
done
timeout -k 10 420 python benchmarks/vlm_rate.py > $O/vlm.log 2>&1
s=$?; echo "vlm exit $s"; tail -1 $O/vlm.log
exit $s
