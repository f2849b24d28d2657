#!/usr/bin/env bash
# Headline bench + kernel-level profile with idle-gap attribution (TAG names the output dir)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/r2_head${TAG:+_$TAG}"; mkdir -p "$O"
export PYTHONUNBUFFERED=1
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
  s=$?; echo "pytest exit $s"; tail -3 $O/pytest.log; [ $s -ne 0 ] && exit $s
fi
timeout -k 10 420 python bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS:-} --out $O/bench.json > $O/bench.log 2>&1
s=$?; echo "bench exit $s"; cat $O/bench.json; [ $s -ne 0 ] && exit $s
[ -n "${NOPROF:-}" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 ${BENCH_ARGS:-} > "$O/prof.log" 2>&1
s=$?; echo "prof exit $s"
python3 "$R/scripts/summarize_prof.py" "$O/raw" > "$O/kernels.txt" 2>&1
head -14 "$O/kernels.txt"; tail -16 "$O/kernels.txt"
rm -rf "$O/raw"
exit $s
