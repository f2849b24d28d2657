#!/bin/bash
# PMC pass over the prefill kernels (v2 by default; V1=1 for the 16x16 kernel)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2_pv2_pmc${V1:+_v1}; mkdir -p $O
[ -n "$V1" ] && export NGA_PREFILL_V1=1
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS} \
  -d $O -o pmc --output-format csv -- python3 $R/benchmarks/kernel_bench.py --only prefill --iters 3 > $O/run.log 2>&1
s=$?; tail -3 $O/run.log; exit $s
