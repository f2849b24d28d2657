#!/bin/bash
# Round 4: skinny GEMM configs (4/8 waves, deeper stages), counter list, one PMC pass
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_skinny2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "skinny or splitk" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 600 python -u benchmarks/skinny_gemm.py --ms 128,256,512 --all > $O/sweep.jsonl 2>&1 || { tail -20 $O/sweep.jsonl; exit 1; }
grep '"lib_us"' $O/sweep.jsonl | cut -c1-400
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 benchmarks/skinny_one.py --shape o --m 256 --cfg 1 --split 4 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
find $O/kt -name "*stats*" | head
