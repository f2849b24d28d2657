#!/usr/bin/env bash
# DePlot / Pix2Struct: GPU numerics test, then the chart-to-table rate (hipGraph vs eager decode)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/deplot; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_pix2struct.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -3 $O/pytest.log; [ $s -ne 0 ] && exit $s
timeout -k 10 300 python benchmarks/deplot_rate.py --images 128 --batch 32 --max-tokens 128 --out $O/rate_graph.json > $O/rate_graph.log 2>&1
s=$?; echo "rate exit $s"; tail -1 $O/rate_graph.log; [ $s -ne 0 ] && exit $s
timeout -k 10 300 python benchmarks/deplot_rate.py --images 128 --batch 32 --max-tokens 128 --no-graph --out $O/rate_eager.json > $O/rate_eager.log 2>&1
s=$?; echo "eager exit $s"; tail -1 $O/rate_eager.log
exit $s
