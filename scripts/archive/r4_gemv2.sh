#!/bin/bash
# Round 4: GEMV in the model (gate/up SwiGLU + LM head at 1-4 rows): end-to-end test, decode latency
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_gemv2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -k "gemv or skinny_gemm_path" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
for b in 1 2 4; do
  for sk in 0 1; do
    NGA_SKINNY=$sk timeout -k 10 240 python -u benchmarks/decode_step.py --batch $b --ctx 1350 > $O/b${b}_sk$sk.json 2> $O/b${b}_sk$sk.err || { tail -10 $O/b${b}_sk$sk.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b${b}_sk$sk.json'));print('batch $b skinny+gemv $sk', d['step_ms'], d['eff_TBps'])"
  done
done
