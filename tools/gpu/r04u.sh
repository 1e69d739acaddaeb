#!/bin/bash
# round 4: point taps in the quad separable up pass -- bloom GPU tests, interleaved A/B against the quad
# kernel without them (and the one-pixel kernel) at 1920x1080 and 1280x720
set -u
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || exit 1
for r in 1 2 3; do for v in pix nopoint point; do
  if [ $v = pix ]; then export BH_BLOOM_NO_SEPQ=1; else unset BH_BLOOM_NO_SEPQ; fi
  L=black_hole_ray_marching_amd/libbh_render.so; [ $v = nopoint ] && L=tools/variants/sepq_nopoint.so
  BH_LIB=$L timeout -k 10 120 python tools/bench_bloom.py --width 1920 --height 1080 --steps 50 --schedule auto > $O/ab1920_${v}_$r.log 2>&1 || exit 1
  BH_LIB=$L timeout -k 10 120 python tools/bench_bloom.py --width 1280 --height 720 --steps 50 --schedule auto > $O/ab1280_${v}_$r.log 2>&1 || exit 1
done; done
