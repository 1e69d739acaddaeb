#!/bin/bash
# round 4: the paired downsamples with their 16 source words gathered first -- bloom GPU tests, interleaved
# A/B against one pass per downsample at 1920x1080 and 4096x2048, kernel trace; then the sticky A/B (r04y)
set -u
O=gpurun_out/r04g2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || exit 1
for r in 1 2 3; do for v in nodown2 base; do
  unset BH_BLOOM_NO_DOWN2
  [ $v = nodown2 ] && export BH_BLOOM_NO_DOWN2=1
  timeout -k 10 120 python tools/bench_bloom.py --width 1920 --height 1080 --steps 50 --schedule auto > $O/ab1920_${v}_$r.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_bloom.py --width 4096 --height 2048 --steps 50 --schedule auto > $O/ab4096_${v}_$r.log 2>&1 || exit 1
done; done
unset BH_BLOOM_NO_DOWN2
timeout -k 10 120 python tools/bench_bloom.py --width 1280 --height 720 --steps 50 --schedule auto > $O/b1280.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace1920 -o run -- python tools/bench_bloom.py --width 1920 --height 1080 --steps 20 --schedule auto > $O/trace1920.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace4096 -o run -- python tools/bench_bloom.py --width 4096 --height 2048 --steps 20 --schedule auto > $O/trace4096.log 2>&1 || exit 1
bash tools/gpu/r04y.sh > $O/r04y.log 2>&1 || exit 1
