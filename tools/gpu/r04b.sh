#!/bin/bash
# round 4: kernel trace of the 1920x1080 and 1280x720 bloom chains (general fused schedule)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04b
for s in "1920 1080" "1280 720"; do
  set -- $s
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r04b/bloom_$1 -o run -- python tools/bench_bloom.py --width $1 --height $2 --steps 20 --warmup 3 > gpurun_out/r04b/bloom_$1.log 2>&1 || exit 1
done
