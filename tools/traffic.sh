#!/bin/bash
# HBM traffic of bench.py's roofline kernel: two PMC passes (FETCH_SIZE, WRITE_SIZE — they cannot
# share a pass), each its own rocprofv3 run with no trace domain, over the kbench case that launches
# the same kernel at the same shape.  Writes profiles/<round>_traffic.json for bench.py.
# usage (on the GPU box): bash tools/traffic.sh r01 "attn L1 self" "flash_attn_kernel<40"
set -o pipefail
R=$GRAFT_REPO_ROOT; ROUND=$1; CASE=$2; KERN=$3
OUT=$R/gpurun_out/traffic_$ROUND; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp KB_PATHS=${KB_PATHS:-v2}
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/p$i -o p -- python3 $R/tools/kbench.py "$CASE" \
    > $OUT/p$i.log 2>&1 || { echo "pmc pass $c failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_traffic.py $OUT "$KERN" $R/gpurun_out/${ROUND}_traffic.json "kbench case '$CASE'"
