#!/bin/bash
# Warm-up cause (frame series incl. hot start), rank 0's work at N=2/4/8 (strong + config4 frames),
# self-launched 2-rank rehearsal with gather verification.
set -u
O=gpurun_out/r02j; mkdir -p $O
timeout -k 10 200 python -u tools/frame_series.py > $O/frame_series.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/probe_rank0.py --n 2,4,8 --frame 4096x2048 > $O/rank0_strong.log 2>&1 || exit 12
timeout -k 10 300 python -u tools/probe_rank0.py --n 8 --frame 8192x4096 > $O/rank0_config4.log 2>&1 || exit 13
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --verify-gather --steps 24 --warmup 16 > $O/rehearsal2.log 2>&1 || exit 14
echo done
