#!/bin/bash
# round 4: raw-word staging of the quad up pass's 28 / 40 tiles (BH_BLOOM_SEPQ_RAW) -- bloom GPU tests with
# both raw, interleaved A/B (0 / 2 / 3) at 1920x1080 and 1280x720
set -u
O=gpurun_out/r04raw; mkdir -p $O
BH_BLOOM_SEPQ_RAW=3 timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom_raw3.log 2>&1 || exit 1
for r in 1 2 3; do for v in 0 2 3; do
  export BH_BLOOM_SEPQ_RAW=$v
  timeout -k 10 120 python tools/bench_bloom.py --width 1920 --height 1080 --steps 50 --schedule auto > $O/ab1920_raw${v}_$r.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_bloom.py --width 1280 --height 720 --steps 50 --schedule auto > $O/ab1280_raw${v}_$r.log 2>&1 || exit 1
done; done
