#!/usr/bin/env bash
# One rocprofv3 kernel-trace profile (name, timeout, cmd...) given in $PROFS; keeps the summary only.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/prof"
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw_$name" -o run -- "$@" > "$O/$name.log" 2>&1
  local s=$?
  echo "$name exit $s"; grep '^{' "$O/$name.log" | tail -1
  python3 "$R/scripts/summarize_prof.py" "$O/raw_$name" > "$O/${name}_kernels.txt" 2>&1
  head -25 "$O/${name}_kernels.txt"
  rm -rf "$O/raw_$name"
  return $s
}
$PROFS
