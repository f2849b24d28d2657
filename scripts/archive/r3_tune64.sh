#!/usr/bin/env bash
# Tune the Llama-3-8B projection GEMMs at M = 320..4352 step 64 (the 256-multiples are in the
# shipped table already) on top of the shipped table, then sweep layer time vs M with it.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
O="$R/gpurun_out/${1:-r3_tune64}"; mkdir -p "$O"
cp "$R/nv_genai_amd/assets/tunableop/gemm_gfx950.csv" "$O/gemm_gfx950.csv"
MS=$(python3 -c "print(','.join(str(m) for m in range(320, 4353, 64) if m % 256))")
timeout -k 10 1000 python3 -u "$R/scripts/tune_gemms.py" --decode "" --prefill "$MS" --max-ms ${TUNE_MS:-400} --iters ${TUNE_ITERS:-60} --out "$O/gemm_gfx950.csv" > "$O/tune.log" 2>&1 || exit $?
NGA_GEMM_TABLE="$O/gemm_gfx950.csv" timeout -k 10 200 python3 -u "$R/benchmarks/gemm_sweep.py" --ms "1024,1088,1152,1216,1280,1344,1408,1472,1536,1600,1664,1728,1792" --tuned > "$O/sweep_tuned.log" 2>&1 || exit $?
