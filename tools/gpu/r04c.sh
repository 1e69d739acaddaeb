#!/bin/bash
# round 4: the general fused bloom chain with fused epilogues -- parity first, then timings, kernel trace,
# PMC; A/B of the quad kernels' padded tile strides (fs0: unpadded, fs1: padded = the build)
set -u
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || exit 1
for s in "1920 1080" "1280 720" "4096 2048"; do
  set -- $s
  timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --steps 50 >> $O/bloom.log 2>&1 || exit 1
done
for r in 1 2; do for v in bloom_fs0 bloom_fs1; do
  BH_LIB=tools/variants/$v.so timeout -k 10 120 python tools/bench_bloom.py --steps 50 > $O/ab_${v}_$r.log 2>&1 || exit 1
done; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace1920 -o run -- python tools/bench_bloom.py --width 1920 --height 1080 --steps 20 --warmup 3 > $O/trace1920.log 2>&1 || exit 1
OUT=r04c/pmc1920 timeout -k 10 300 tools/gpu/bloom_pmc.sh 1920 1080 > $O/pmc.log 2>&1 || exit 1
OUT=r04c/pmc4096 timeout -k 10 300 tools/gpu/bloom_pmc.sh 4096 2048 > $O/pmc4096.log 2>&1 || exit 1
