export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/rank_emulate.py --world 8 --ab-fused 10 --steps 20 > gpurun_out/ab_fused_w8.log 2>&1 || exit 1
tail -3 gpurun_out/ab_fused_w8.log
timeout -k 10 300 python3 tools/rank_emulate.py --world 4 --ab-fused 10 --steps 20 > gpurun_out/ab_fused_w4.log 2>&1 || exit 1
tail -3 gpurun_out/ab_fused_w4.log
