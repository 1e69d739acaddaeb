#!/bin/bash
# round 4: software-pipelined texel reads in the separable up pass -- bloom GPU tests, interleaved A/B at
# 1920x1080 and 1280x720
set -u
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || exit 1
for r in 1 2 3; do for v in sep_pipe0 sep_pipe1; do
  BH_LIB=tools/variants/$v.so timeout -k 10 120 python tools/bench_bloom.py --width 1920 --height 1080 --steps 50 > $O/ab1920_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 120 python tools/bench_bloom.py --width 1280 --height 720 --steps 50 > $O/ab1280_${v}_$r.log 2>&1 || exit 1
done; done
