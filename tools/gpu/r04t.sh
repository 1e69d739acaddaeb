#!/bin/bash
# round 4: kernel traces of the bloom chains at 4096x2048 (fused) and 1920x1080 (general, quad form)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r04t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for s in "4096 2048" "1920 1080"; do
  set -- $s
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace$1 -o run -- python tools/bench_bloom.py --width $1 --height $2 --steps 20 --warmup 3 --schedule auto > $O/trace$1.log 2>&1 || exit 1
done
