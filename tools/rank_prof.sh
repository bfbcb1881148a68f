#!/bin/bash
# Emulated rank-0 step of an N-way frame-sharded run (tools/rank_emulate.py: 16/N frames, the
# motion modules on all 16 frames of HW/N positions after the re-shard, every collective a
# same-size device copy), timed, then under rocprofv3 and summarised per step
# (tools/prof_summary.py) into gpurun_out/rank_w<N>.txt.  WORLDS (default "8 4 2").
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for w in ${WORLDS:-8 4 2}; do
  timeout -k 10 300 python3 $R/tools/rank_emulate.py --world $w --chunks 1 --comm copy --steps 20 > $R/gpurun_out/rank_w$w.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/rank_w$w.log
  [ -n "$NO_PROF" ] && continue
  RAW=/tmp/vd_rank_w$w; rm -rf $RAW
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $RAW -o run -- python3 $R/tools/rank_emulate.py --world $w --chunks 1 --comm copy --steps 6 > $R/gpurun_out/rank_prof_w$w.log 2>&1) || exit 1
  python3 $R/tools/prof_summary.py $(find $RAW -name "*kernel_trace.csv" | head -1) > $R/gpurun_out/rank_w$w.txt || exit 1
  head -1 $R/gpurun_out/rank_w$w.txt
done
