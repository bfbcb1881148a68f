#!/bin/bash
# rocprofv3 kernel trace + stats of the DiT bench (tools/dit_bench.py), summarised per step.
mkdir -p gpurun_out/ditprof
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ditprof -o run -- python3 $R/tools/dit_bench.py --steps 4 --warmup 1 $DIT_ARGS > $R/gpurun_out/ditprof/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 $R/gpurun_out/ditprof/bench.log
[ $rc -ne 0 ] && exit $rc
f=$(find $R/gpurun_out/ditprof -name "*kernel_trace.csv" | head -1)
python3 $R/tools/prof_summary.py $f > $R/gpurun_out/ditprof/step_breakdown.txt
cat $R/gpurun_out/ditprof/step_breakdown.txt | head -50
