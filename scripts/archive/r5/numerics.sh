#!/bin/bash
# Round 5: the generation smoke checks (lp_tol 0.25) and the teacher-forced logit comparisons
# with their printed worst errors (-s), then the whole GPU suite
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/r5_numerics
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -s -v -p no:cacheprovider --timeout 200 --timeout-method thread \
  "tests/test_engine_gpu.py::test_step_graphs_equal_eager_steps" \
  "tests/test_engine_gpu.py::test_step_graphs_headline_gqa_4096_bucket" \
  "tests/test_engine_gpu.py::test_skinny_gemm_path_matches_library_path" \
  "tests/test_engine_gpu.py::test_teacher_forced_graph_logits_match_eager" \
  "tests/test_engine_gpu.py::test_teacher_forced_headline_gqa_4096_bucket" \
  "tests/test_kernels_gpu.py::test_skinny_table_production_shapes" > $out/numerics.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|worst|delta|smoke|passed|failed" $out/numerics.log | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/archive/r5/full.sh r5_numerics_full
