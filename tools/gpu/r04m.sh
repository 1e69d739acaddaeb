#!/bin/bash
# round 4: the far-field level of the root-free step -- GPU suite, its wave-step share, interleaved A/B
# against the kept root-free form alone (skipv2)
set -u
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || exit 1
BH_LIB=tools/variants/diag.so timeout -k 10 120 python tools/diag_slow.py > $O/diag.log 2>&1 || exit 1
for r in 1 2 3; do for v in skipv2 far; do
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-extra > $O/h_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu --no-extra > $O/c2_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --config 1 --steps 20 --warmup 5 --no-cpu --no-extra > $O/c1_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --config 5 --frames-per-launch 1 --steps 100 --warmup 20 --no-cpu --no-extra > $O/c5f1_${v}_$r.log 2>&1 || exit 1
done; done
