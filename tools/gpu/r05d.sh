#!/bin/bash
# round 5: the quad separable pass's per-axis shared texels (BH_BLOOM_SEPQ_AXIS, build switch) and the Y
# epilogue's in-block fix (BH_BLOOM_NO_FIX, runtime switch) -- bloom parity on the GPU, per-wave timelines of
# the quad launches (probe_bloom_phases), interleaved A/B of the chain
set -u
source tools/gpu/outdir.sh r05 d
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || { tail -30 $O/pytest_bloom.log; exit 1; }
tail -2 $O/pytest_bloom.log
for s in "1920 1080" "1280 720"; do
  set -- $s
  BH_LIB=tools/variants/bphase.so timeout -k 10 120 python tools/probe_bloom_phases.py --width $1 --height $2 >> $O/phases.log 2>&1 || exit 1
done
for rep in 1 2 3; do
  for v in main nofix noaxis; do
    for s in "1920 1080" "1280 720"; do
      set -- $s
      L=black_hole_ray_marching_amd/libbh_render.so; E=""
      if [ $v = noaxis ]; then L=tools/variants/$v.so; fi
      if [ $v = nofix ]; then E="BH_BLOOM_NO_FIX=1"; fi
      env $E BH_LIB=$L timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --schedule auto --steps 200 2>/dev/null | sed "s/^/$v /" >> $O/ab.log || exit 1
    done
  done
done
cut -c1-200 $O/ab.log
