#!/bin/bash
# round 4: GPU suite with the root-free step (sdf_skip) as default, its wave-step share, A/B skip0 vs
# skip1 (headline, config 2, config 5 at one frame per launch), bloom timings + stride A/B, phases, bloom trace
set -u
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || exit 1
BH_LIB=tools/variants/diag.so timeout -k 10 120 python tools/diag_slow.py > $O/diag.log 2>&1 || exit 1
cp black_hole_ray_marching_amd/libbh_render.so tools/variants/skip1.so
for r in 1 2 3; do for v in skip0 skip1; do
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu > $O/h_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu > $O/c2_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --config 5 --frames-per-launch 1 --steps 100 --warmup 20 --no-cpu > $O/c5f1_${v}_$r.log 2>&1 || exit 1
done; done
for s in "1920 1080" "1280 720" "4096 2048"; do
  set -- $s
  timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --steps 50 >> $O/bloom.log 2>&1 || exit 1
done
for r in 1 2; do for v in bloom_fs0 bloom_fs1 bloom_fs2 bloom_fs3; do
  BH_LIB=tools/variants/$v.so timeout -k 10 120 python tools/bench_bloom.py --steps 50 > $O/ab_${v}_$r.log 2>&1 || exit 1
done; done
BH_LIB=tools/variants/phases.so timeout -k 10 120 python tools/probe_phases.py > $O/phases.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace1920 -o run -- python tools/bench_bloom.py --width 1920 --height 1080 --steps 20 --warmup 3 > $O/trace1920.log 2>&1 || exit 1
