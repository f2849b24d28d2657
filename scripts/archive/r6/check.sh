#!/bin/bash
# Round 6: smoke(), the packed-upload / TP / TP=8 GPU tests, and the 256 x 1,400 decode step
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_check}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python -u -m pytest tests/test_tp8_rehearsal_gpu.py tests/test_tp_gpu.py tests/test_kernels_gpu.py -k "tp or packed or custom" -q -p no:cacheprovider --timeout 600 --timeout-method thread -rf > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 > $out/decode256.json 2> $out/decode256.err || { tail -20 $out/decode256.err; exit 1; }
tail -1 $out/decode256.json
