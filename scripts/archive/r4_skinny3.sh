#!/bin/bash
# Round 4: skinny GEMM layout variants at M = 256 (plain, K rotation, packed W, packed W + x) and
# the headline-GQA step-graph tests
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4_skinny3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "skinny or splitk" > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
for v in "plain:" "krot:--krot 1" "wpack:--wpack" "wxpack:--wpack --xpack" "wxpack_krot:--wpack --xpack --krot 1"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u benchmarks/skinny_gemm.py --ms 64,256 --shapes o,qkv,down,gate_up --cfgs 0,1,2,3,10,13,16 $a > $O/sweep_$n.jsonl 2>&1 || { tail -20 $O/sweep_$n.jsonl; exit 1; }
  echo "== $n"; grep '"lib_us"' $O/sweep_$n.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); b=r['best_gemm']; print(r['shape'], r['M'], 'lib', r['lib_us'], 'best', b['cfg'], b['split'], b['gemm_us'], b['total_us'])"
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "gqa_4096" > $O/gqa.txt 2>&1; echo "gqa exit $?"; grep -E "PASS|FAIL|Error|assert" $O/gqa.txt | head -20
