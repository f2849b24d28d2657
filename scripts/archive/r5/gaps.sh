#!/bin/bash
# Round 5: launch gaps inside the decode step's hipGraph (256 x 1,400), and the same step with
# kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1)
set -o pipefail
cd "$(dirname "$0")/../.."
R=$PWD
out=gpurun_out/r5_gaps
mkdir -p $out
timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 32 > $out/decode_base.json 2> $out/decode_base.err || { tail -20 $out/decode_base.err; exit 1; }
tail -1 $out/decode_base.json
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 32 > $out/decode_devkernarg.json 2> $out/decode_devkernarg.err || { tail -20 $out/decode_devkernarg.err; exit 1; }
tail -1 $out/decode_devkernarg.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/$out/raw -o run -- python3 $R/benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 > $R/$out/prof.log 2>&1 || { tail -20 $R/$out/prof.log; exit 1; }
python3 $R/scripts/archive/r5/graph_gaps.py $R/$out/raw > $R/$out/gaps.txt 2>&1
rm -rf $R/$out/raw
cat $R/$out/gaps.txt
