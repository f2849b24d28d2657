#!/bin/bash
# Round 5: chosen (cfg, split) pairs of the decode-shape GEMM at M = 256 with their consumers
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_probe
mkdir -p $out
run() { timeout -k 10 120 python -u benchmarks/skinny_probe.py "$@" >> $out/probe.jsonl 2>&1 || { tail -20 $out/probe.jsonl; exit 1; }; }
: > $out/probe.jsonl
run --shape gate_up --m 256 --pairs 13:1,16:1,17:1,18:1,21:1,35:1,36:1,37:1,38:1,35:2,36:2,38:2,17:2,18:2,20:2,33:2,34:2,19:2,21:2,17:3,18:3,13:2,12:2
run --shape down --m 256 --pairs 13:8,16:8,12:16,35:16,36:16,36:8,38:16,17:8,17:16,18:8,18:16,33:16,34:16,19:16,21:16,20:16
run --shape o --m 256 --pairs 1:4,10:4,13:8,35:8,36:8,36:16,17:8,17:16,18:8,18:16,19:8,22:8,24:4,21:8
run --shape qkv --m 256 --pairs 16:4,13:4,35:4,36:4,36:8,17:8,18:8,17:4,18:4,19:4,21:4,22:4,24:2,33:8
run --shape lm_head --m 256 --pairs 12:1,11:1,17:1,18:1,19:1,21:1,35:1,36:1
cat $out/probe.jsonl
