#!/bin/bash
# round 5: a shard's per-tile cost against the one-GPU frame's: N = 8 with rank 0's
# calibrated share (0.55) at 64 and 256 frames per launch, the tile interleave at the tile (the default) and
# at 2x2 / 4x4 tile super-blocks (BH_PARTITION_SB, A/B), and the whole frame in the packed layout (--n 1)
set -u
source tools/gpu/outdir.sh r05 c
for D in 64 256; do
  timeout -k 10 200 python tools/probe_rank0.py --n 1 --D $D --it 6 >> $O/rank0.jsonl 2> $O/rank0.err || exit 1
  for sb in 1 2 4; do
    BH_PARTITION_SB=$sb timeout -k 10 200 python tools/probe_rank0.py --n 8 --D $D --root-ratio 0.55 --it 6 --tag sb$sb >> $O/rank0.jsonl 2>> $O/rank0.err || exit 1
  done
done
