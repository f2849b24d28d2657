#!/bin/bash
# Wave-per-row RMSNorm + the DMA decode policy (rebuilt launcher): kernel tests, engine tests,
# norm / decode kernel benches.
set -o pipefail
O=gpurun_out/r3_norm_decode; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_families_gpu.py -x -v --timeout 200 --timeout-method thread > $O/test_kernels.log 2>&1 || { grep -n "Error\|assert" $O/test_kernels.log | head -20; tail -5 $O/test_kernels.log; exit 1; }
tail -2 $O/test_kernels.log
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread > $O/test_engine.log 2>&1 || { grep -n "Error\|assert" $O/test_engine.log | head -20; tail -5 $O/test_engine.log; exit 1; }
tail -2 $O/test_engine.log
timeout -k 10 200 python benchmarks/kernel_bench.py --only norm > $O/kb_norm.json 2> $O/kb_norm.err || { tail -20 $O/kb_norm.err; exit 1; }
cat $O/kb_norm.json
timeout -k 10 300 python benchmarks/kernel_bench.py --only decode > $O/kb_decode.json 2> $O/kb_decode.err || { tail -20 $O/kb_decode.err; exit 1; }
cat $O/kb_decode.json
timeout -k 10 600 python bench.py --workload agent --steps 2 --warmup 1 > $O/agent_70b_tp1.json 2> $O/agent.err || { tail -20 $O/agent.err; exit 1; }
cat $O/agent_70b_tp1.json
