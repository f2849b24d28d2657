#!/bin/bash
# Prefill attention: numerics of both kernels, then timings of each at serving shapes
set -o pipefail
mkdir -p gpurun_out/r2_pv2
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "prefill or varlen" > gpurun_out/r2_pv2/test.log 2>&1 || { tail -30 gpurun_out/r2_pv2/test.log; exit 1; }
tail -3 gpurun_out/r2_pv2/test.log
timeout -k 10 200 python -u benchmarks/kernel_bench.py --only prefill > gpurun_out/r2_pv2/bench.json 2> gpurun_out/r2_pv2/bench.err || exit 1
cat gpurun_out/r2_pv2/bench.json
