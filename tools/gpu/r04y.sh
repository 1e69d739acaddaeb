#!/bin/bash
# round 4: the sticky root-free test (after a tested slow step, the next takes the roots untested) A/B
set -u
O=gpurun_out/r04y; mkdir -p $O
BH_LIB=tools/variants/sticky.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/pytest_sticky.log 2>&1 || exit 1
for r in 1 2 3; do for v in cur sticky; do
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-extra > $O/h_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu --no-extra > $O/c2_${v}_$r.log 2>&1 || exit 1
done; done
