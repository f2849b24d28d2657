#!/bin/bash
# Round 6: the 32-deep-stage decode-shape GEMM tiles (cfgs 17-21): numerics of every cfg, then
# each llama3-8b projection at M = 128-256 with its consumer, every (cfg, split) printed
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_bk32}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "skinny" -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $out/pytest_skinny.log 2>&1 || { tail -30 $out/pytest_skinny.log; exit 1; }
tail -2 $out/pytest_skinny.log
timeout -k 10 900 python benchmarks/skinny_table.py --model llama3-8b --shapes gate_up,down,o,qkv --ms 128,192,224,256 --all --out $out/table.json > $out/sweep.jsonl 2> $out/sweep.err || { tail -20 $out/sweep.err; exit 1; }
grep '"lib_us"' $out/sweep.jsonl
