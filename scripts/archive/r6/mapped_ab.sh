#!/bin/bash
# Round 6: the step upload as one scatter kernel reading mapped host staging (no copy dispatch):
# the probe (host time behind a busy stream, device time per upload, data check), the kernel
# and engine GPU tests, then interleaved against per-buffer copies (NGA_PACKED_UPLOAD=0): the
# 256 x 1,400 decode step and the headline (8 steps)
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_h2d}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
timeout -k 10 200 python -u scripts/dev/h2d_probe.py > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
tail -1 $out/probe.log > $out/probe.json
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
for pk in 1 0 1 0; do
  NGA_PACKED_UPLOAD=$pk timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 > $out/decode_pk$pk.json 2> $out/decode_pk$pk.err || { tail -20 $out/decode_pk$pk.err; exit 1; }
  echo "packed=$pk $(tail -1 $out/decode_pk$pk.json)"
done
for i in 1 2; do
  for pk in 1 0; do
    NGA_PACKED_UPLOAD=$pk timeout -k 10 400 python bench.py --steps 8 --warmup 2 > $out/bench_pk${pk}_$i.json 2> $out/bench_pk${pk}_$i.err || { tail -20 $out/bench_pk${pk}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_pk${pk}_$i.json'));print('packed=$pk', d['value'], d['p50_latency_ms'], d['host_step_ms']['all']['launch'], d['gpu_step_timing']['between_steps_ms'])"
  done
done
