#!/bin/bash
# Final-build evidence: every single-GPU config with the CPU leg (parity + cpu_baseline), the
# predicted strong-scaling curve (shards at 8 frames per launch), rank 0's work, a 2-rank orbit
# rehearsal (self-launched, gather verified per frame's camera).
set -u
O=gpurun_out/r02x; mkdir -p $O
bash tools/configs.sh > $O/configs.log 2>&1 || exit 11
cp -r gpurun_out/configs $O/ || true
timeout -k 10 400 python -u tools/probe_inflight.py --modes batch --frames 4096x2048,8192x4096 --shards 1,2,4,8 --depths 1,8 > $O/inflight.log 2>&1 || exit 12
timeout -k 10 300 python -u tools/probe_rank0.py --n 2,4,8 --rows 64 --frame 4096x2048 > $O/rank0_strong.log 2>&1 || exit 13
timeout -k 10 300 python -u tools/probe_rank0.py --n 8 --rows 64 --frame 8192x4096 > $O/rank0_config4.log 2>&1 || exit 14
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --verify-gather --camera-path orbit --steps 24 --warmup 16 > $O/rehearsal2_orbit.log 2>&1 || exit 15
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 3 --verify-gather --fmt bgra8 --steps 12 --warmup 8 > $O/rehearsal3_bgra8.log 2>&1 || exit 16
echo done
