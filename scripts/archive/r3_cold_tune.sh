#!/bin/bash
# Cold-operand re-tune of the M = 256 / 512 projection GEMMs (rotating buffer > MALL), then the
# decode-only step with the shipped table vs the re-tuned one, interleaved.
set -o pipefail
O=gpurun_out/r3_cold; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python scripts/retune_cold.py --ms 256,512 --rotating-mb 1024 --out $O/gemm_cold.csv > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
python scripts/retune_cold.py --merge --out $O/gemm_cold.csv >> $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -2 $O/tune.log
diff <(sort nv_genai_amd/assets/tunableop/gemm_gfx950.csv) <(sort $O/gemm_cold.csv) > $O/table.diff; cat $O/table.diff | head -40
for r in 1 2; do
  timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1350 --steps 32 > $O/ds_base_r$r.json 2> $O/ds_base_r$r.err || { tail -5 $O/ds_base_r$r.err; exit 1; }
  NGA_GEMM_TABLE=$O/gemm_cold.csv timeout -k 10 300 python benchmarks/decode_step.py --batch 256 --ctx 1350 --steps 32 > $O/ds_cold_r$r.json 2> $O/ds_cold_r$r.err || { tail -5 $O/ds_cold_r$r.err; exit 1; }
  echo "base: $(cat $O/ds_base_r$r.json)"; echo "cold: $(cat $O/ds_cold_r$r.json)"
done
