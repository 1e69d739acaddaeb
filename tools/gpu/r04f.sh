#!/bin/bash
# round 4: the GPU suite (op 12/13 self-tests of the rsq-seeded reciprocal, bloom general chain),
# bloom timings + stride A/B, a headline line, wave-phase probe, bloom trace
set -u
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_crmath.py > $O/crmath.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 150 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || exit 1
for s in "1920 1080" "1280 720" "4096 2048"; do
  set -- $s
  timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --steps 50 >> $O/bloom.log 2>&1 || exit 1
done
for r in 1 2; do for v in bloom_fs0 bloom_fs1 bloom_fs2 bloom_fs3; do
  BH_LIB=tools/variants/$v.so timeout -k 10 120 python tools/bench_bloom.py --steps 50 > $O/ab_${v}_$r.log 2>&1 || exit 1
done; done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu > $O/headline.log 2>&1 || exit 1
BH_LIB=tools/variants/phases.so timeout -k 10 120 python tools/probe_phases.py > $O/phases.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace1920 -o run -- python tools/bench_bloom.py --width 1920 --height 1080 --steps 20 --warmup 3 > $O/trace1920.log 2>&1 || exit 1
