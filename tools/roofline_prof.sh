#!/bin/bash
# The roofline object's evidence at this tree, in one GPU call (VERDICT r2 "make the roofline
# reproducible"):
#  1. rocprofv3 --kernel-trace --stats over a short bench.py run with the DEFAULT roofline call
#     (10 warm-up + 20 timed launches after the step loop): tools/prof_summary.py prints the
#     step breakdown and the roofline kernel's average over exactly those 20 launches, next to
#     the bench line the same run printed (avg_launch_ms) -> <round>_roofline_trace.txt;
#  2. FETCH_SIZE and WRITE_SIZE, each its own PMC pass over `bench.py --roofline-only` (the same
#     time_attention call, nothing else launched) -> <round>_traffic.json (gfx950 corrections);
#  3. SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE pass over the same -> <round>_mfma_busy.json.
# Both JSONs carry kernel_src_hash; bench.py reads only summaries whose hash matches its tree.
# usage (GPU box): bash tools/roofline_prof.sh r03a
set -o pipefail
R=$GRAFT_REPO_ROOT; ROUND=${1:-r03}
OUT=/tmp/vd_roof_$ROUND; rm -rf $OUT; mkdir -p $OUT  # raw traces stay on the box (gpurun copies back < 64 MiB)
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-nocfg > $OUT/bench_prof.json 2> $OUT/bench_prof.log \
  || { echo "trace run failed"; tail -5 $OUT/bench_prof.log; exit 1; }
TR=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
ST=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
{ python3 $R/tools/prof_summary.py $TR; echo; echo "bench line of the same (profiled) run:";
  python3 -c "import json,sys; r=json.load(open(sys.argv[1]))['roofline']; print('  roofline.avg_launch_ms', r['avg_launch_ms'], 'achieved', r['achieved'], 'TF/s frac', r['frac'], 'stress', r['stress'])" $OUT/bench_prof.json; } \
  > $R/gpurun_out/${ROUND}_roofline_trace.txt || exit 1
cp $ST $R/gpurun_out/${ROUND}_kernel_stats.csv
cp $OUT/bench_prof.json $R/gpurun_out/${ROUND}_bench_prof.json
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/p$i -o p -- python3 $R/bench.py --roofline-only \
    > $OUT/p$i.log 2>&1 || { echo "pmc pass $c failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_traffic.py $OUT "flash40_kernel<true>" $R/gpurun_out/${ROUND}_traffic.json \
  "bench.py --roofline-only (the step's own L1 operands: 5 in-model + 10 warm + 20 timed launches, 32 images)" || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA --output-format csv -d $OUT/mb -o p -- \
  python3 $R/bench.py --roofline-only > $OUT/mb.log 2>&1 || { echo "mfma pass failed"; tail -5 $OUT/mb.log; exit 1; }
python3 $R/tools/mfma_busy.py $OUT/mb $R/gpurun_out/${ROUND}_mfma_busy.json > $R/gpurun_out/${ROUND}_mfma_busy.txt || exit 1
cat $R/gpurun_out/${ROUND}_roofline_trace.txt | tail -4; cat $R/gpurun_out/${ROUND}_traffic.json; cat $R/gpurun_out/${ROUND}_mfma_busy.txt
