#!/bin/bash
# ABI v5 (device frame table beyond 32 frames per launch): the multi-frame + partition GPU tests, then
# frames per launch 32..256 on configs 1 and 2 and 32/64 on the headline (interleaved, 2 reps).
set -u
O=gpurun_out/r02aw; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -k "render_frames or partition or prepared" --timeout 300 --timeout-method thread > $O/pytest_frames.log 2>&1 || exit 10
tail -2 $O/pytest_frames.log
for rep in 1 2; do
  for D in 32 64 128 256; do
    timeout -k 10 200 python -u bench.py --config 1 --no-cpu --steps 512 --warmup 512 --frames-per-launch $D > $O/c1_D${D}_r$rep.log 2>&1 || exit 11
    tail -1 $O/c1_D${D}_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1 D$D r$rep', d['ms_per_step'], d['kernel']['ms_per_frame'], d['roofline']['frac'])"
  done
  for D in 32 64 128; do
    timeout -k 10 200 python -u bench.py --config 2 --no-cpu --steps 256 --warmup 256 --frames-per-launch $D > $O/c2_D${D}_r$rep.log 2>&1 || exit 12
    tail -1 $O/c2_D${D}_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 D$D r$rep', d['ms_per_step'], d['kernel']['ms_per_frame'], d['roofline']['frac'])"
  done
  for D in 32 64; do
    timeout -k 10 200 python -u bench.py --no-cpu --steps 128 --warmup 256 --frames-per-launch $D > $O/c3_D${D}_r$rep.log 2>&1 || exit 13
    tail -1 $O/c3_D${D}_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 D$D r$rep', d['ms_per_step'], d['kernel']['ms_per_frame'], d['roofline']['frac'])"
  done
done
echo done
