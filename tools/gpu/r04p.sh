#!/bin/bash
# round 4: a shard's per-tile cost against the frames per launch (the capped rays' chains vs the launch)
set -u
O=gpurun_out/r04p; mkdir -p $O
for D in 16 32 64; do
  timeout -k 10 300 python tools/probe_rank0.py --n 8 --D $D --rows 64 --root-ratio 1,0.55 --transport rgbm14 --it 6 >> $O/rank0_D.jsonl 2>> $O/rank0_D.err || exit 1
done
timeout -k 10 300 python tools/probe_rank0.py --n 1 --D 16 --rows 64 --root-ratio 1 --transport rgbm14 --it 6 >> $O/rank0_D.jsonl 2>> $O/rank0_D.err || exit 1
