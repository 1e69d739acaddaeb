#!/bin/bash
# round 4: does alternating the render launches over two streams (one launch's tail overlapping the next
# launch's start) bring a shard's per-tile cost back to the one-GPU frame's?
set -u
O=gpurun_out/r04l; mkdir -p $O
for rs in 1 2; do
  timeout -k 10 300 python tools/probe_rank0.py --n 1,2,8 --D 16 --rows 64 --root-ratio 1 --transport rgbm14 --it 8 --render-streams $rs >> $O/rank0_streams.jsonl 2>> $O/rank0_streams.err || exit 1
done
timeout -k 10 300 python tools/probe_rank0.py --n 8 --D 16 --rows 64 --root-ratio 0.55,0.6 --transport rgbm14 --it 8 --render-streams 2 >> $O/rank0_streams.jsonl 2>> $O/rank0_streams.err || exit 1
