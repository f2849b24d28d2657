#!/bin/bash
# Round 6: gate/up at M = 256 on the 224 x 128 tile (cfg 27, shipped table) vs the 256 x 128 tile
# (cfg 13, NGA_SKINNY_TABLE=scripts/archive/r6/skinny_table_cfg13.json), in the step: production
# table numerics, then interleaved on one box the 256 x 1,400 decode step and the headline
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_bn224_ab}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
OLD=$PWD/scripts/archive/r6/skinny_table_cfg13.json
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "production or skinny" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for v in new old new old; do
  if [ $v = old ]; then export NGA_SKINNY_TABLE=$OLD; else unset NGA_SKINNY_TABLE; fi
  timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 > $out/decode_$v.json 2> $out/decode_$v.err || { tail -20 $out/decode_$v.err; exit 1; }
  echo "$v $(tail -1 $out/decode_$v.json)"
done
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export NGA_SKINNY_TABLE=$OLD; else unset NGA_SKINNY_TABLE; fi
    timeout -k 10 400 python bench.py --steps 8 --warmup 2 > $out/bench_${v}_$i.json 2> $out/bench_${v}_$i.err || { tail -20 $out/bench_${v}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$out/bench_${v}_$i.json'));print('$v', d['value'], d['p50_latency_ms'])"
  done
done
