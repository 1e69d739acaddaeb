#!/bin/bash
# A/B: 16 vs 32 frames per launch (BH_MAX_FRAMES 32) on every single-GPU config and the N=8 shards.
set -u
O=gpurun_out/r02ao; mkdir -p $O
for C in 1 2 3 5; do
  for rep in 1 2; do
    for D in 16 32; do
      timeout -k 10 200 python -u bench.py --config $C --no-cpu --steps 160 --warmup 320 --frames-per-launch $D > $O/c${C}_D${D}_r$rep.log 2>&1 || exit 1
      tail -1 $O/c${C}_D${D}_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c$C D$D r$rep', d['ms_per_step'], d['kernel']['ms_per_frame'], d['roofline']['frac'])"
    done
  done
done
timeout -k 10 400 python -u tools/probe_inflight.py --frames 4096x2048,8192x4096 --shards 8 --depths 16,32,16,32 --modes batch > $O/inflight_shards.log 2>&1 || exit 2
echo done
