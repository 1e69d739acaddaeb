#!/bin/bash
# round 4: the quad form of the separable up pass (up_sepq_kernel) -- bloom GPU tests, interleaved A/B
# against the one-pixel kernel (BH_BLOOM_NO_SEPQ=1) at 1920x1080 and 1280x720, and its PMC at 1920x1080
set -u
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || exit 1
for r in 1 2 3; do for v in pix quad; do
  if [ $v = pix ]; then export BH_BLOOM_NO_SEPQ=1; else unset BH_BLOOM_NO_SEPQ; fi
  timeout -k 10 120 python tools/bench_bloom.py --width 1920 --height 1080 --steps 50 > $O/ab1920_${v}_$r.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_bloom.py --width 1280 --height 720 --steps 50 > $O/ab1280_${v}_$r.log 2>&1 || exit 1
done; done
unset BH_BLOOM_NO_SEPQ
OUT=r04q/bloom_pmc_1920 bash tools/gpu/bloom_pmc.sh 1920 1080 > $O/bloom_pmc.log 2>&1 || exit 1
