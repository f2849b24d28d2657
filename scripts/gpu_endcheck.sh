#!/bin/bash
# What the round driver runs at round end, on this tree: smoke(), the whole GPU test suite, and
# bench.py at the driver's configuration (20 steps, 5 warm-up). Usage: gpu_endcheck.sh [out-name]
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-endcheck}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf -s > $out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $out/pytest_gpu.log | head -20; tail -4 $out/pytest_gpu.log; exit 1; }
grep -E "teacher-forced rows|greedy smoke" $out/pytest_gpu.log | tail -4
tail -1 $out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));print('bench', d['value'], d['p50_latency_ms'], d['p50_ttft_ms'], d['prefix_cache']['hit_share'], d['gpu_step_timing'])"
