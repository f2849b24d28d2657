#!/bin/bash
# Decode-only step at the headline's steady state (256 rows, ~1,350-token contexts): engine
# step / bare graph replay time and a per-kernel breakdown of the replayed graphs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/r3_decode_step"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python "$R/benchmarks/decode_step.py" --batch 256 --ctx 1350 --steps 32 > "$O/decode_step.json" 2> "$O/decode_step.err" || { tail -20 "$O/decode_step.err"; exit 1; }
cat "$O/decode_step.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw" -o run -- \
  python3 "$R/benchmarks/decode_step.py" --batch 256 --ctx 1350 --steps 32 > "$O/prof.log" 2>&1 || { tail -20 "$O/prof.log"; exit 1; }
python3 "$R/scripts/summarize_prof.py" "$O/raw" > "$O/kernels.txt" 2>&1
rm -rf "$O/raw"
head -30 "$O/kernels.txt" | cut -c1-150
timeout -k 10 200 python "$R/benchmarks/gemm_sweep.py" --tuned --ms 64,128,256,320,512,768 > "$O/gemm_small_m.log" 2>&1 || { tail -20 "$O/gemm_small_m.log"; exit 1; }
cat "$O/gemm_small_m.log"
timeout -k 10 200 python "$R/benchmarks/kernel_bench.py" --only norm > "$O/kb_norm.json" 2> "$O/kb_norm.err" || { tail -20 "$O/kb_norm.err"; exit 1; }
cat "$O/kb_norm.json"
