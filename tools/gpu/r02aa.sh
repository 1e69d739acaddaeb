#!/bin/bash
# Weighted partitions: GPU tests, rank-0 balance probe, N=2 / N=3 rehearsals through the bench.
set -u
O=gpurun_out/r02aa; mkdir -p $O
true
timeout -k 10 500 python -u tools/probe_rank0.py --n 2,4,8 --root-ratio 1,auto,0.7 --frame 4096x2048 > $O/rank0_strong.log 2>&1 || exit 12
timeout -k 10 400 python -u tools/probe_rank0.py --n 8 --root-ratio 1,auto,0.7 --frame 8192x4096 > $O/rank0_config4.log 2>&1 || exit 13
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --verify-gather --steps 24 --warmup 16 > $O/rehearsal2.log 2>&1 || exit 14
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 3 --verify-gather --fmt bgra8 --camera-path orbit --steps 12 --warmup 8 > $O/rehearsal3.log 2>&1 || exit 15
echo done
