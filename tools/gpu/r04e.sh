#!/bin/bash
# round 4: rank 0 / other-rank probes for the N>1 model (RGBM14 vs RGBM transport, 16 vs 32 frames per launch)
set -u
O=gpurun_out/r04e; mkdir -p $O
for D in 16 32; do
  timeout -k 10 300 python tools/probe_rank0.py --n 2,4,8 --D $D --rows 64 --root-ratio auto,1 --transport rgbm14 --it 8 >> $O/rank0.jsonl 2> $O/rank0_$D.err || exit 1
done
timeout -k 10 300 python tools/probe_rank0.py --n 8 --D 16 --rows 64 --root-ratio auto --transport rgbm --it 8 >> $O/rank0.jsonl 2>> $O/rank0_rgbm.err || exit 1
