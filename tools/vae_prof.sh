#!/bin/bash
# VAE decode: bench line, then a rocprofv3 kernel-trace/stats pass of the same command.
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python tools/vae_bench.py ${VAE_ARGS:-} > gpurun_out/vae_bench.json 2> gpurun_out/vae_bench.log || exit 1
cat gpurun_out/vae_bench.json
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_vae
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_vae -o run -- python3 $GRAFT_REPO_ROOT/tools/vae_bench.py --reps 1 --cpu-frames 0 > $GRAFT_REPO_ROOT/gpurun_out/vae_prof.log 2>&1 || exit 1
head -12 $GRAFT_REPO_ROOT/gpurun_out/prof_vae/run_kernel_stats.csv | cut -c1-160
