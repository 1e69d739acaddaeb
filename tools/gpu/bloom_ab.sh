#!/bin/bash
# Bloom parity, then an interleaved A/B of the chain (default vs the env arm given as $1, e.g.
# BH_BLOOM_NO_YDOWN2=1) at the three display sizes; `notest` as $2 skips the parity tests:
#   bash tools/gpu/bloom_ab.sh ARM [notest]        -> gpurun_out/r06/bloom/<time>/
set -u -o pipefail
source tools/gpu/outdir.sh r06 bloom
ARM=${1:-BH_BLOOM_NO_YDOWN2=1}
if [ "${2:-}" != notest ]; then
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || { tail -30 $O/pytest_bloom.log; exit 1; }
tail -1 $O/pytest_bloom.log
fi
for rep in 1 2 3; do
  for v in main arm; do
    for s in "1920 1080" "1280 720" "4096 2048"; do
      set -- $s
      if [ $v = main ]; then E=""; else E="$ARM"; fi
      env $E timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --schedule auto --steps 200 2>>$O/ab.err | sed "s/^/$v /" >> $O/ab.log || exit 1
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
for k in sorted(r): print(k, ["%.5f" % x for x in r[k]], "min %.5f" % min(r[k]))
PY
