#!/bin/bash
# Round 6 baseline: the whole GPU test suite, then the driver's bench configuration and the
# 256 x 1,400 decode step on this box.
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_base}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $out/pytest_gpu.log 2>&1
rc=$?
tail -8 $out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('bench', d['value'],d['p50_latency_ms'],d['p50_ttft_ms'],d['prefix_cache'])"
timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 > $out/decode256.json 2> $out/decode256.err || { tail -20 $out/decode256.err; exit 1; }
tail -2 $out/decode256.json
exit $rc
