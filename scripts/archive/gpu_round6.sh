#!/usr/bin/env bash
# pytest -m gpu (pinned-buffer race fix), then tune the projection GEMMs into the shipped table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s"; tail -4 gpurun_out/pytest_gpu.log
if [ $s -ne 0 ] && [ $s -ne 1 ]; then exit $s; fi
timeout -k 10 900 python scripts/tune_gemms.py > gpurun_out/tune.log 2>&1
s=$?; echo "tune exit $s"; tail -3 gpurun_out/tune.log
cp nv_genai_amd/assets/tunableop/gemm_gfx950.csv gpurun_out/gemm_gfx950.csv
exit $s
