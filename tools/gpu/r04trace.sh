#!/bin/bash
# round 4, final build: kernel traces of the bloom chain at 1920x1080 and 4096x2048
set -u
O=gpurun_out/r04trace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace1920 -o run -- python tools/bench_bloom.py --width 1920 --height 1080 --steps 20 --schedule auto > $O/trace1920.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace4096 -o run -- python tools/bench_bloom.py --width 4096 --height 2048 --steps 20 --schedule auto > $O/trace4096.log 2>&1 || exit 1
