#!/bin/bash
# Prepared launches (FrameBatch): the new GPU test, then every config at 32 frames per launch.
set -u
O=gpurun_out/r02aq; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "prepared or render_frames" > $O/pytest.log 2>&1 || exit 11
for C in 1 2 3 5; do
  for rep in 1 2; do
    timeout -k 10 200 python -u bench.py --config $C --no-cpu --steps 160 --warmup 320 > $O/c${C}_r$rep.log 2>&1 || exit 1
    tail -1 $O/c${C}_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c$C r$rep', d['ms_per_step'], d['kernel']['ms_per_frame'], d['kernel']['avg_ms'], d['roofline']['frac'], d['roofline']['traffic'])"
  done
done
echo done
