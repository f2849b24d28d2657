#!/usr/bin/env bash
# Tune the projection GEMMs at the steady-state mixed-step token counts (256-aligned,
# 512..2304) on top of the shipped table, then sweep default vs tuned at those M.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/tune"
mkdir -p "$O"
cp "$R/nv_genai_amd/assets/tunableop/gemm_gfx950.csv" "$O/gemm_gfx950.csv"
MS=${MS:-512,768,1024,1280,1536,1792,2048,2304}
timeout -k 10 900 python3 -u "$R/scripts/tune_gemms.py" --decode "" --prefill "$MS" --max-ms ${TUNE_MS:-1000} --iters ${TUNE_ITERS:-100} --out "$O/gemm_gfx950.csv" > "$O/tune.log" 2>&1 || exit $?
tail -3 "$O/tune.log"
timeout -k 10 300 python3 -u "$R/benchmarks/gemm_sweep.py" --ms "$MS" > "$O/sweep_default.log" 2>&1 || exit $?
NGA_GEMM_TABLE="$O/gemm_gfx950.csv" timeout -k 10 300 python3 -u "$R/benchmarks/gemm_sweep.py" --ms "$MS" --tuned > "$O/sweep_tuned.log" 2>&1 || exit $?
paste <(grep '^{' "$O/sweep_default.log" | python3 -c "import sys,json; [print(json.loads(l)['M'], json.loads(l)['layer_us']) for l in sys.stdin]") <(grep '^{' "$O/sweep_tuned.log" | python3 -c "import sys,json; [print(json.loads(l)['layer_us']) for l in sys.stdin]")
