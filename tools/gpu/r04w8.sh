#!/bin/bash
# round 4: a waves-per-EU bound for the 8-tap bloom kernels (BH_BLOOM_WPE 7: up2 72 VGPRs, 7 waves;
# 8: 64 VGPRs with 8 spilled) -- bloom GPU tests with both, interleaved A/B at 4096x2048 and 1920x1080
set -u
O=gpurun_out/r04w8; mkdir -p $O
for v in bw7 bw8; do
  BH_LIB=tools/variants/$v.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom_$v.log 2>&1 || exit 1
done
for r in 1 2 3; do for v in base bw7 bw8; do
  L=tools/variants/$v.so; [ $v = base ] && L=black_hole_ray_marching_amd/libbh_render.so
  BH_LIB=$L timeout -k 10 120 python tools/bench_bloom.py --width 4096 --height 2048 --steps 50 --schedule auto > $O/ab4096_${v}_$r.log 2>&1 || exit 1
  BH_LIB=$L timeout -k 10 120 python tools/bench_bloom.py --width 1920 --height 1080 --steps 50 --schedule auto > $O/ab1920_${v}_$r.log 2>&1 || exit 1
done; done
