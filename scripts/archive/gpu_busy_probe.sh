#!/usr/bin/env bash
# GPU busy % during the headline bench without a profiler attached: rocm-smi GPU use sampled
# every 0.25 s next to a plain bench run (the kernel-trace profiler slows the host's launches,
# so its busy fraction understates an unprofiled run)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; cd "$R"
O="$R/gpurun_out/busy"; mkdir -p "$O"
( while true; do echo "$(date +%s.%N) $(rocm-smi --showuse 2>/dev/null | grep -o 'GPU use (%): *[0-9]*' | grep -o '[0-9]*$' | head -1)"; sleep 0.25; done ) > "$O/smi.txt" 2>&1 &
P=$!
timeout -k 10 400 python bench.py --steps 8 --warmup 2 --out $O/bench.json > $O/bench.log 2>&1
s=$?
kill $P 2>/dev/null
echo "bench exit $s"; cat $O/bench.json
python3 - "$O/smi.txt" <<'PY'
import sys
rows = [l.split() for l in open(sys.argv[1]) if len(l.split()) == 2]
v = [float(b) for _, b in rows]
n = len(v)
tail = v[int(0.45 * n): int(0.95 * n)]          # the timed steady state (after setup + warm-up)
print("samples", n, "steady-state mean GPU use %", round(sum(tail) / max(1, len(tail)), 1),
      "min", min(tail) if tail else None, "share of samples < 95%:", round(sum(1 for x in tail if x < 95) / max(1, len(tail)), 3))
PY
exit $s
