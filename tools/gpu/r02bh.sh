#!/bin/bash
# A/B: tile-schedule workgroups of 1 wave (wg1) vs 4 waves (wg4) over the single-GPU configs, interleaved.
set -u
O=gpurun_out/r02bh; mkdir -p $O
timeout -k 10 500 bash tools/ab_interleaved.sh 3 "--steps 64 --warmup 64" wg4 wg1 > $O/c3.log 2>&1 || exit 1
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--config 2 --steps 128 --warmup 64" wg4 wg1 > $O/c2.log 2>&1 || exit 2
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--config 5 --steps 64 --warmup 64" wg4 wg1 > $O/c5.log 2>&1 || exit 3
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--config 1 --steps 1024 --warmup 512" wg4 wg1 > $O/c1.log 2>&1 || exit 4
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--frames-per-launch 1 --steps 64 --warmup 64" wg4 wg1 > $O/c3_D1.log 2>&1 || exit 5
for f in c3 c2 c5 c1 c3_D1; do echo "== $f"; cat $O/$f.log; done
