#!/bin/bash
# round 5: rounds of resident blocks in the quad separable pass -- raw-word tiles for the 28 / 40 footprints
# (BH_BLOOM_SEPQ_RAW, runtime) and 8 waves per SIMD (build variant wpe8): bloom parity, per-wave timelines, A/B
set -u
source tools/gpu/outdir.sh r05 e
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || { tail -30 $O/pytest_bloom.log; exit 1; }
tail -1 $O/pytest_bloom.log
# the variant library's bloom parity at its best setting (a quick subset)
BH_LIB=tools/variants/wpe8.so BH_BLOOM_SEPQ_RAW=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bloom.py -k "1920 or 1280" > $O/pytest_bloom_wpe8.log 2>&1 || { tail -30 $O/pytest_bloom_wpe8.log; exit 1; }
tail -1 $O/pytest_bloom_wpe8.log
for s in "1920 1080" "1280 720"; do
  set -- $s
  BH_LIB=tools/variants/bphase.so timeout -k 10 120 python tools/probe_bloom_phases.py --width $1 --height $2 | sed "s/^/main /" >> $O/phases.log 2>&1 || exit 1
  BH_LIB=tools/variants/bphase8.so BH_BLOOM_SEPQ_RAW=2 timeout -k 10 120 python tools/probe_bloom_phases.py --width $1 --height $2 | sed "s/^/wpe8raw2 /" >> $O/phases.log 2>&1 || exit 1
done
for rep in 1 2 3; do
  for v in main mainraw2 wpe8 wpe8raw2 wpe8raw3; do
    for s in "1920 1080" "1280 720"; do
      set -- $s
      L=black_hole_ray_marching_amd/libbh_render.so; R=0
      case $v in wpe8*) L=tools/variants/wpe8.so;; esac
      case $v in *raw2) R=2;; *raw3) R=3;; esac
      BH_BLOOM_SEPQ_RAW=$R BH_LIB=$L timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --schedule auto --steps 100 2>/dev/null | sed "s/^/$v /" >> $O/ab.log || exit 1
    done
  done
done
python3 - $O/ab.log <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    v, j = l.split(" ", 1); j = json.loads(j); d[(v, j["width"])].append(j["avg_ms"])
for k, x in sorted(d.items()): print(k, [round(a, 5) for a in x], round(sum(x) / len(x), 5))
PY
