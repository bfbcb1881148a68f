#!/bin/bash
# rocprofv3 kernel trace of bench.py at each frame count in $FRAMES (default "16 2"),
# summarised per step by tools/prof_summary.py into gpurun_out/breakdown_f<F>.txt
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for f in ${FRAMES:-16 2}; do
  # raw traces stay on the box (/tmp): gpurun copies gpurun_out/ back only below 64 MiB
  RAW=/tmp/vd_prof_f$f; rm -rf $RAW
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $RAW -o run -- python3 $GRAFT_REPO_ROOT/bench.py --frames $f --steps 6 --warmup 2 --no-cpu-baseline --no-nocfg --attn-reps ${ATTN_REPS:-2} > $GRAFT_REPO_ROOT/gpurun_out/prof_f$f.log 2>&1 || exit 1
  python3 $GRAFT_REPO_ROOT/tools/prof_summary.py $(find $RAW -name "*kernel_trace.csv" | head -1) > $GRAFT_REPO_ROOT/gpurun_out/breakdown_f$f.txt || exit 1
  cp $(find $RAW -name "*kernel_stats.csv" | head -1) $GRAFT_REPO_ROOT/gpurun_out/kernel_stats_f$f.csv
  head -3 $GRAFT_REPO_ROOT/gpurun_out/breakdown_f$f.txt
done
