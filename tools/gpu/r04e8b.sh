#!/bin/bash
# round 4: the raw 60 tile at stride 64 (LDS 28 -> 24 KiB: 6 blocks per CU) with and without a 6-waves
# bound (80 VGPRs, spills) -- bloom GPU tests with both, interleaved A/B with e8 and the base build
set -u
O=gpurun_out/r04e8b; mkdir -p $O
for v in e8fs64 e8fs64w6; do
  BH_LIB=tools/variants/$v.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py -k "bitexact or general or graph" > $O/pytest_bloom_$v.log 2>&1 || exit 1
done
for r in 1 2 3; do for v in bbase e8 e8fs64 e8fs64w6; do
  BH_LIB=tools/variants/$v.so timeout -k 10 120 python tools/bench_bloom.py --width 1920 --height 1080 --steps 50 --schedule auto > $O/ab1920_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 120 python tools/bench_bloom.py --width 1280 --height 720 --steps 50 --schedule auto > $O/ab1280_${v}_$r.log 2>&1 || exit 1
done; done
