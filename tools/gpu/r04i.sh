#!/bin/bash
# round 4: which form of the root-free test schedules best: v1 (compares + ballot), v2 (fma slack, select),
# v3 (fma slack, fcmp lane mask) against skip0 (no skip), interleaved
set -u
O=gpurun_out/r04i; mkdir -p $O
for r in 1 2 3; do for v in skip0 skipv1 skipv2 skipv3; do
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-extra > $O/h_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu --no-extra > $O/c2_${v}_$r.log 2>&1 || exit 1
done; done
