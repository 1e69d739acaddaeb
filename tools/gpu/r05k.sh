#!/bin/bash
# round 5: the final pass at 7 blocks per CU -- the alpha table in constant memory (1 KiB less LDS per block)
# with a 7-waves bound (variant alut7) or without it (alut6): parity of the variants, interleaved A/B
set -u -o pipefail
source tools/gpu/outdir.sh r05 k
for v in alut7 alut6; do
  BH_LIB=tools/variants/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bloom.py -k "1920 or 1280 or any_alpha or 1366" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
for rep in 1 2 3; do
  for v in main alut7 alut6; do
    L=black_hole_ray_marching_amd/libbh_render.so; if [ $v != main ]; then L=tools/variants/$v.so; fi
    for s in "1920 1080" "1280 720" "4096 2048"; do
      set -- $s
      BH_LIB=$L timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --schedule auto --steps 200 2>>$O/ab.err | sed "s/^/$v /" >> $O/ab.log || exit 1
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
