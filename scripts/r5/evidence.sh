#!/bin/bash
# Round 5: numerics evidence + the whole GPU suite, then the large-M GEMM probe
set -o pipefail
cd "$(dirname "$0")/../.."
bash scripts/r5/numerics.sh
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc    # anything but test failures: stop here
bash scripts/r5/large_m.sh | tail -30
exit $rc
