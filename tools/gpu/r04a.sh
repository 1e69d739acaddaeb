#!/bin/bash
# round 4: VALU/transcendental issue ubench, bloom parity (general fused chain) + timings
set -u
mkdir -p gpurun_out/r04a
timeout -k 10 60 tools/ubench/trans_mix > gpurun_out/r04a/trans_mix.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bloom.py > gpurun_out/r04a/pytest_bloom.log 2>&1 || exit 1
for s in "1920 1080" "1280 720" "4096 2048"; do
  set -- $s
  timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --steps 50 >> gpurun_out/r04a/bloom.log 2>&1 || exit 1
done
