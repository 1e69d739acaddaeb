#!/bin/bash
# No-surface kernel instantiation (SF = 0): parity suites, then config 1 at the auto frames per launch
# (256) with the bench's oracle leg, and D = 32 / 256 timings.
set -u
O=gpurun_out/r02ax; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 10
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --config 1 > $O/c1_default.log 2>&1 || exit 11
tail -1 $O/c1_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1 default', d['config']['frames_per_launch'], d['ms_per_step'], d['kernel']['ms_per_frame'], d['kernel']['name'], d['roofline']['frac'], d['parity']['bit_exact'], d['parity']['timed_format_bit_exact'])"
for rep in 1 2; do
  for D in 32 256; do
    timeout -k 10 200 python -u bench.py --config 1 --no-cpu --steps 512 --warmup 512 --frames-per-launch $D > $O/c1_D${D}_r$rep.log 2>&1 || exit 12
    tail -1 $O/c1_D${D}_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1 D$D r$rep', d['ms_per_step'], d['kernel']['ms_per_frame'], d['roofline']['frac'])"
  done
done
echo done
