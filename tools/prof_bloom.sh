#!/bin/bash
# Kernel trace of the bloom chain (tools/bench_bloom.py) -> gpurun_out/prof_bloom_TAG/
set -u
TAG=${1:-x}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_bloom_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_bloom.py --steps 20 --warmup 2 > "$OUT/trace.log" 2>&1 || exit 1
echo ok
