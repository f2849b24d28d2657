#!/usr/bin/env bash
# Tune the projection GEMMs at M = 4608..5376 on top of the shipped table, then A/B the headline
# at mixed-step prefill budgets 4096 / 4864 / 5120 with that table.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
O="$R/gpurun_out/tune_big"; mkdir -p "$O"
cp "$R/nv_genai_amd/assets/tunableop/gemm_gfx950.csv" "$O/gemm_gfx950.csv"
MS=4608,4864,5120,5376
timeout -k 10 600 python3 -u "$R/scripts/tune_gemms.py" --decode "" --prefill "$MS" --max-ms 1000 --iters 100 --out "$O/gemm_gfx950.csv" > "$O/tune.log" 2>&1 || exit $?
NGA_GEMM_TABLE="$O/gemm_gfx950.csv" timeout -k 10 300 python3 -u "$R/benchmarks/gemm_sweep.py" --ms "4096,4352,$MS" --tuned > "$O/sweep_tuned.log" 2>&1 || exit $?
grep '^{' "$O/sweep_tuned.log" | python3 -c "import sys,json; [print(json.loads(l)['M'], json.loads(l)['layer_us']) for l in sys.stdin]"
export NGA_GEMM_TABLE="$O/gemm_gfx950.csv"
i=0
for t in 4096 4864 5120 4096 4864 5120; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --mixed-prefill-tokens $t --out $O/bench_${t}_r$i.json > $O/bench_${t}_r$i.log 2>&1
  s=$?; [ $s -ne 0 ] && { echo "bench $t exit $s"; tail -5 $O/bench_${t}_r$i.log; exit $s; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'QPS', d['value'], 'p50', d['p50_latency_ms'], 'ttft', d['p50_ttft_ms'])" $O/bench_${t}_r$i.json $t
done
