#!/bin/bash
# Round 6: a 224 x 128 skinny tile (cfg 27: one wave column of 224 weight rows, 4 token waves)
# for gate/up + SwiGLU, whose 128 x 2 blocks fill the 256 CUs (the shipped 256 x 128 tile
# makes 224): every-cfg numerics, then the table tuner's timing with consumers at M 192-320
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_bn224}
mkdir -p $out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "every_cfg or skinny" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 400 python benchmarks/skinny_table.py --shapes gate_up --ms 192,224,256,320 --cfgs 13,27,16,0 --all --out $out/table.json > $out/table.jsonl 2> $out/table.err || { tail -20 $out/table.err; exit 1; }
cat $out/table.jsonl
