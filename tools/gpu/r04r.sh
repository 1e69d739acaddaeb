#!/bin/bash
# round 4: the quad separable up pass with parity-ordered plan entries -- bloom GPU tests, A/B at 1920x1080
# and 1280x720 against the one-pixel kernel, PMC at 1920x1080
set -u
O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || exit 1
for r in 1 2 3; do for v in pix quad stream; do
  if [ $v = pix ]; then export BH_BLOOM_NO_SEPQ=1; else unset BH_BLOOM_NO_SEPQ; fi
  L=black_hole_ray_marching_amd/libbh_render.so; [ $v = stream ] && L=tools/variants/sepq_stream.so
  BH_LIB=$L timeout -k 10 120 python tools/bench_bloom.py --width 1920 --height 1080 --steps 50 > $O/ab1920_${v}_$r.log 2>&1 || exit 1
  BH_LIB=$L timeout -k 10 120 python tools/bench_bloom.py --width 1280 --height 720 --steps 50 > $O/ab1280_${v}_$r.log 2>&1 || exit 1
done; done
BH_LIB=tools/variants/sepq_stream.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom_stream.log 2>&1 || exit 1
unset BH_BLOOM_NO_SEPQ
OUT=r04r/bloom_pmc_1920 bash tools/gpu/bloom_pmc.sh 1920 1080 > $O/bloom_pmc.log 2>&1 || exit 1
