#!/bin/bash
# Round 5: bench.py TP=2 rehearsal on one GPU (ranks share the device, gloo groups, IPC
# collectives, pipelined graphed steps); stacks dumped every 60 s if it stalls
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/${1:-r5_tp2}
shift
mkdir -p $out
NGA_TRACE_CAPTURE=1 NGA_STACK_DUMP_S=60 timeout -k 10 400 python bench.py --gpus 2 --tp 2 --allow-shared-devices "$@" > $out/tp2.json 2> $out/tp2.err || { grep -v "amdgpu.ids\|socket.cpp\|Gloo" $out/tp2.err | tail -80; exit 1; }
python -c "import json;d=json.load(open('$out/tp2.json'));print('tp2', d['value'], d['unpipelined_steps'], d['step_graphs']['timed_graph_steps'], d['devices']['ranks'][0].get('custom_all_reduce'))"
