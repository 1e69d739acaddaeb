#!/bin/bash
# A/B: ballot of the bare r^2 < 1 compare (no predicate materialisation) vs the current step.
set -u
mkdir -p gpurun_out/r02as
timeout -k 10 900 bash tools/ab_interleaved.sh 3 "--steps 160 --warmup 320" base ballot > gpurun_out/r02as/headline.log 2>&1 || exit 11
timeout -k 10 600 bash tools/ab_interleaved.sh 3 "--config 2 --steps 160 --warmup 320" base ballot > gpurun_out/r02as/c2.log 2>&1 || exit 12
timeout -k 10 600 bash tools/ab_interleaved.sh 2 "--config 5 --frames-per-launch 1 --steps 100 --warmup 200" base ballot > gpurun_out/r02as/c5_D1.log 2>&1 || exit 13
echo done
