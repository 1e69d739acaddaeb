#!/bin/bash
# A/B: packed vs scalar tail step, interleaved rounds on one box.
set -u
O=gpurun_out/r02g; mkdir -p $O
tools/ab_interleaved.sh 3 "--steps 96 --warmup 96" tailpk tailscalar > $O/ab_c3_D8.log 2>&1 || exit 11
tools/ab_interleaved.sh 3 "--steps 96 --warmup 96 --frames-per-launch 1" tailpk tailscalar > $O/ab_c3_D1.log 2>&1 || exit 12
tools/ab_interleaved.sh 3 "--steps 96 --warmup 96 --frames-per-launch 1 --max-iters 1000 --camera C" tailpk tailscalar > $O/ab_c5_D1.log 2>&1 || exit 13
echo done
