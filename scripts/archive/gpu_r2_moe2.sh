set -u
bash scripts/gpu_r2_moe.sh && ABLS="0" TOKS=256,1536,4096 bash scripts/gpu_r2_moe_abl.sh
