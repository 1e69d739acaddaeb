#!/bin/bash
# The N>1 path on the prepared-launch build: 2-rank orbit and 3-rank BGRA8 rehearsals (gather-verified),
# the one-rank RCCL dry run (test + full size).
set -u
O=gpurun_out/r02au; mkdir -p $O
BH_BENCH_REHEARSAL=1 timeout -k 10 400 python -u bench.py --gpus 2 --verify-gather --camera-path orbit --steps 24 --warmup 8 > $O/rehearsal2_orbit.log 2>&1 || exit 11
BH_BENCH_REHEARSAL=1 timeout -k 10 400 python -u bench.py --gpus 3 --verify-gather --fmt bgra8 --steps 16 --warmup 8 > $O/rehearsal3_bgra8.log 2>&1 || exit 12
timeout -k 10 300 python -u -m pytest tests/test_bench_launch.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest_dry.log 2>&1 || exit 13
timeout -k 10 300 python -u bench.py --rccl-dry-run --verify-gather --steps 48 --warmup 96 > $O/bench_dry_full.log 2>&1 || exit 14
for f in rehearsal2_orbit rehearsal3_bgra8 bench_dry_full; do tail -1 $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['n_gpus'], d.get('world_size'), d.get('backend'), d['gather_verified_bit_exact'], d['ms_per_step'])"; done
echo done
