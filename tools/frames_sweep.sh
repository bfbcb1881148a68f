#!/bin/bash
# Per-GPU step time at F/N frames (the compute share of one rank under N-way frame
# sharding, without the collectives): bench.py --frames f on one GPU.
mkdir -p gpurun_out
for f in ${FRAMES:-16 8 4 2}; do
  timeout -k 10 200 python bench.py --frames $f --steps 10 --warmup 2 --no-cpu-baseline --no-nocfg --attn-reps 2 \
    > gpurun_out/frames_$f.json 2> gpurun_out/frames_$f.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/frames_$f.json')); print('frames', $f, d['ms_per_step'], 'ms/step')"
done
