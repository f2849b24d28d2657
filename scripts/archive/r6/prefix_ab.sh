#!/bin/bash
# (runs against the tree with scripts/archive/decode_prefix_pass.patch applied; the pass is not shipped)
# Round 6: shared-prefix decode pass (decode_prefix_kernel). GPU tests of the kernels and the
# engine, then interleaved on one box against NGA_DECODE_PREFIX=0: the 256 x 1,400 decode step
# with a 133-token shared prompt head (the RAG template), and the headline (8 steps)
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_prefix}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_kernel_forms.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
for pf in 1 0 1 0; do
  NGA_DECODE_PREFIX=$pf timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 --shared-prefix 133 > $out/decode_pf$pf.json 2> $out/decode_pf$pf.err || { tail -20 $out/decode_pf$pf.err; exit 1; }
  echo "prefix=$pf $(tail -1 $out/decode_pf$pf.json)"
done
for i in 1 2; do
  for pf in 1 0; do
    NGA_DECODE_PREFIX=$pf timeout -k 10 400 python bench.py --steps 8 --warmup 2 > $out/bench_pf${pf}_$i.json 2> $out/bench_pf${pf}_$i.err || { tail -20 $out/bench_pf${pf}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_pf${pf}_$i.json'));print('prefix=$pf', d['value'], d['p50_latency_ms'], d['shared_prefix_pass'])"
  done
done
