#!/bin/bash
# Round 6: the GPU suite, then the packed step upload (one copy + one scatter kernel) against
# per-buffer copies (NGA_PACKED_UPLOAD=0), interleaved on one box: headline (8 steps) and the
# 256 x 1,400 decode step
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_packed}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $out/pytest_gpu.log 2>&1
rc=$?
tail -6 $out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for pk in 1 0; do
    NGA_PACKED_UPLOAD=$pk timeout -k 10 400 python bench.py --steps 8 --warmup 2 > $out/bench_pk${pk}_$i.json 2> $out/bench_pk${pk}_$i.err || { tail -20 $out/bench_pk${pk}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_pk${pk}_$i.json'));print('packed=$pk', d['value'], d['p50_latency_ms'], d['host_step_ms']['all']['launch'], d['gpu_step_timing']['between_steps_ms'])"
  done
done
for pk in 1 0 1 0; do
  NGA_PACKED_UPLOAD=$pk timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 > $out/decode_pk$pk.json 2> $out/decode_pk$pk.err || { tail -20 $out/decode_pk$pk.err; exit 1; }
  echo "packed=$pk $(tail -1 $out/decode_pk$pk.json)"
done
exit $rc
