#!/bin/bash
# round 4: the gather form of the bloom fix-up pass and the paired downsamples -- bloom GPU tests,
# interleaved A/B (base / per-sample fix-up / one pass per downsample) at 1920x1080 and 4096x2048,
# 1280x720, a kernel trace of the 1920x1080 chain
set -u
O=gpurun_out/r04fix; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || exit 1
BH_BLOOM_SEPQ_MIN_BLOCKS=1024 timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py -k bitexact > $O/pytest_bloom_minb.log 2>&1 || exit 1
for r in 1 2 3; do for v in sample nodown2 minb base; do
  unset BH_BLOOM_FIXUP_SAMPLE BH_BLOOM_NO_DOWN2 BH_BLOOM_SEPQ_MIN_BLOCKS
  [ $v = sample ] && export BH_BLOOM_FIXUP_SAMPLE=1
  [ $v = nodown2 ] && export BH_BLOOM_NO_DOWN2=1
  [ $v = minb ] && export BH_BLOOM_SEPQ_MIN_BLOCKS=1024
  timeout -k 10 120 python tools/bench_bloom.py --width 1920 --height 1080 --steps 50 --schedule auto > $O/ab1920_${v}_$r.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_bloom.py --width 4096 --height 2048 --steps 50 --schedule auto > $O/ab4096_${v}_$r.log 2>&1 || exit 1
done; done
unset BH_BLOOM_FIXUP_SAMPLE BH_BLOOM_NO_DOWN2 BH_BLOOM_SEPQ_MIN_BLOCKS
timeout -k 10 120 python tools/bench_bloom.py --width 1280 --height 720 --steps 50 --schedule auto > $O/b1280.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace1920 -o run -- python tools/bench_bloom.py --width 1920 --height 1080 --steps 20 --schedule auto > $O/trace1920.log 2>&1 || exit 1
