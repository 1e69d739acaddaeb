#!/bin/bash
# round 4: the march kernel at 8 waves per SIMD (64 VGPRs, a 20-byte spill) against 7 (66 VGPRs)
set -u
O=gpurun_out/r04w; mkdir -p $O
for r in 1 2 3; do for v in cur wpe8; do
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-extra > $O/h_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu --no-extra > $O/c2_${v}_$r.log 2>&1 || exit 1
done; done
