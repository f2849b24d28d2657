#!/bin/bash
# PMC counters of the 256 x 1,400 decode step (benchmarks/decode_step.py, graph replays): HBM
# bytes per dispatch (FETCH_SIZE / WRITE_SIZE, each in its own pass) and the SQ instruction mix,
# summarised per kernel by scripts/pmc_summary.py. Counters only: kernel trace, no other trace
# domains. Usage: gpu_pmc_step.sh [out-name]
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
out=$R/gpurun_out/${1:-pmc_step}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $out/$name -o run -- \
      python3 $R/benchmarks/decode_step.py --batch 256 --ctx 1400 --steps 4 > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }
  python3 $R/scripts/pmc_summary.py $out/$name decode_attn skinny_gemm Cijk rope_cache rmsnorm sample_kernel > $out/$name.txt 2>&1
  rm -rf $out/$name
}
pass fetch FETCH_SIZE && pass write WRITE_SIZE && pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU
