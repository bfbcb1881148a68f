#!/bin/bash
# GEMM path comparison at the per-rank image counts of 1/2/4/8-way frame sharding.
mkdir -p gpurun_out
for n in ${IMGS_LIST:-32 16 8 4}; do
  KB_IMGS=$n KB_PATHS=${KB_PATHS:-auto,pre6,v6} timeout -k 10 300 python tools/kbench.py "${KB_FILTER:-}" > gpurun_out/kb_imgs$n.log 2>&1 || exit 1
done
