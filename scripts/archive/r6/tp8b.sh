#!/bin/bash
# Round 6: the TP = 8 rehearsal tests (with wake-up stats) + the 8-rank sharded search test,
# then RAG with a TP = 2 replica and its sharded index (searches on the retrieval stream)
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_tp8b}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_tp8_rehearsal_gpu.py -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $out/pytest_tp8.log 2>&1 || { grep -E "PASS|FAIL|Error" $out/pytest_tp8.log | tail; tail -30 $out/pytest_tp8.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $out/pytest_tp8.log | tail -5
GPU_MAX_HW_QUEUES=2 timeout -k 10 600 python bench.py --gpus 2 --tp 2 --sharded-index --allow-shared-devices --steps 2 --warmup 1 --concurrency 64 --kv-cache-fraction 0.1 --out $out/bench_tp2_sharded.json > $out/bench_tp2.log 2>&1 || { tail -30 $out/bench_tp2.log; exit 1; }
python -c "import json;d=json.load(open('$out/bench_tp2_sharded.json'));print('tp2 sharded', d['value'], d['p50_latency_ms'], d['unpipelined_steps'], [r.get('custom_all_reduce',{}).get('timeout_flag') for r in d['devices']['ranks']])"
