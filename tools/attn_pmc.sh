#!/bin/bash
# PMC passes over tools/attn_one.py for each d = 40 attention variant -> gpurun_out/attn_pmc/
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/attn_pmc; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for sel in ${SELS:-2 3}; do
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
             "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/s$sel/p$i -o p -- python3 $R/tools/attn_one.py $sel 3 > $OUT/s${sel}_p$i.log 2>&1 || { echo "sel $sel pass $i failed"; tail -3 $OUT/s${sel}_p$i.log; exit 1; }
  done
done
for sel in ${SELS:-2 3}; do echo "== select $sel"; python3 $R/tools/pmc_summary.py $OUT/s$sel | grep -v "at::native" ; done > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
