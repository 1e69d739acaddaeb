#!/bin/bash
# round 5: the fix-up kernel indexing (32-bit quotients, 24-bit multiplies, unconditional loads;
# tools/variants/prevfix.so = the previous commit) -- bloom parity on the GPU, interleaved A/B of the chain
set -u -o pipefail
source tools/gpu/outdir.sh r05 fixidx
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || { tail -30 $O/pytest_bloom.log; exit 1; }
tail -2 $O/pytest_bloom.log
for rep in 1 2 3; do
  for v in main prevfix; do
    for s in "1920 1080" "1280 720" "4096 2048"; do
      set -- $s
      L=black_hole_ray_marching_amd/libbh_render.so; if [ $v != main ]; then L=tools/variants/$v.so; fi
      BH_LIB=$L timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --schedule auto --steps 200 2>>$O/ab.err | sed "s/^/$v /" >> $O/ab.log || exit 1
    done
  done
done
python3 - $O <<'PY'
import json, sys
from collections import defaultdict
O = sys.argv[1]
r = defaultdict(list)
for l in open(f"{O}/ab.log"):
    v, j = l.split(" ", 1)
    b = json.loads(j); r[(v, b["width"])].append(b["avg_ms"])
for k in sorted(r): print(k, ["%.5f" % x for x in r[k]])
PY
