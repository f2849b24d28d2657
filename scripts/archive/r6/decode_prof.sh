#!/bin/bash
# Round 6: kernel table of the 256 x 1,400 decode step (graph replays)
set -o pipefail
cd "$(dirname "$0")/../../.."
R=$PWD
out=gpurun_out/${1:-r6_decode_prof}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/raw -o run -- python3 $R/benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 16 > $R/$out/prof.log 2>&1 || { tail -20 $R/$out/prof.log; exit 1; }
python3 $R/scripts/summarize_prof.py $R/$out/raw > $R/$out/kernels.txt 2>&1
rm -rf $R/$out/raw
head -32 $R/$out/kernels.txt | cut -c1-160
