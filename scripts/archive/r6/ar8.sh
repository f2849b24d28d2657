#!/bin/bash
# Round 6: why the W = 8 one-GPU engine rehearsal timed out in the custom all-reduce: grid cap
# per call and HIP queues per rank, eager and graph-replayed, 8 ranks on cuda:0
set -o pipefail
cd "$(dirname "$0")/../../.."
out=gpurun_out/${1:-r6_ar8}
mkdir -p $out
export PYTHONUNBUFFERED=1
for v in "--blocks 80" "--blocks 10" "--blocks 80 --queues 2" "--blocks 10 --graph" "--blocks 80 --graph" "--blocks 80 --world 4"; do
  echo "== $v"
  timeout -k 10 240 python scripts/dev/ar8_probe.py $v >> $out/probe.jsonl 2>> $out/probe.err || { echo "rc=$? on $v"; tail -5 $out/probe.err; exit 1; }
  tail -1 $out/probe.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ok'],d['errors'],d['bad'],d['s_per_iter'],d['r0'].get('max_blocks'),d['r0'].get('exc'))"
done
