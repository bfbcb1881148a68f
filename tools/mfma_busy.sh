#!/bin/bash
# MFMA-busy share per kernel family over a short bench.py run (one PMC pass, no trace domains):
# SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs).  -> gpurun_out/mfma_busy.txt
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/mfma_pmc; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA --output-format csv -d $OUT -o p -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-nocfg --attn-reps 3 ${BENCH_ARGS:-} > $OUT/run.log 2>&1 || { tail -5 $OUT/run.log; exit 1; }
python3 $R/tools/mfma_busy.py $OUT $R/gpurun_out/${ROUND:-r01}_mfma_busy.json > $R/gpurun_out/mfma_busy.txt && cat $R/gpurun_out/mfma_busy.txt
