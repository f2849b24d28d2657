#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/r6_bk32b
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "skinny_gemm_every" -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $out/pytest_skinny.log 2>&1 || { tail -30 $out/pytest_skinny.log; exit 1; }
tail -1 $out/pytest_skinny.log
timeout -k 10 600 python benchmarks/skinny_table.py --model llama3-8b --shapes gate_up,down,o --ms 128,256 --cfgs 1,9,10,13,16,20,21,22,23,24,25,26 --all --out $out/table.json > $out/sweep.jsonl 2> $out/sweep.err || { tail -20 $out/sweep.err; exit 1; }
grep '"lib_us"' $out/sweep.jsonl
bash scripts/gpu_busy.sh r6_busy
