#!/bin/bash
# round 5: column strips for the final fix-up (BH_BLOOM_NO_STRIPS: off, runtime switch) -- bloom parity on
# the GPU (with and without), per-wave timelines of the fix-up, interleaved A/B of the chain
set -u -o pipefail
source tools/gpu/outdir.sh r05 strips
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || { tail -30 $O/pytest_bloom.log; exit 1; }
tail -2 $O/pytest_bloom.log
BH_BLOOM_NO_STRIPS=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom_nostrips.log 2>&1 || { tail -30 $O/pytest_bloom_nostrips.log; exit 1; }
tail -2 $O/pytest_bloom_nostrips.log
for v in main nostrips; do
  E=""; if [ $v = nostrips ]; then E="BH_BLOOM_NO_STRIPS=1"; fi
  echo "variant $v" >> $O/phases.log
  env $E BH_LIB=tools/variants/bphase.so timeout -k 10 120 python tools/probe_bloom_phases.py --width 1920 --height 1080 --chains 5 >> $O/phases.log 2>> $O/phases.err || exit 1
done
for rep in 1 2 3; do
  for v in main nostrips; do
    for s in "1920 1080" "1280 720"; do
      set -- $s
      E=""; if [ $v = nostrips ]; then E="BH_BLOOM_NO_STRIPS=1"; fi
      env $E timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --schedule auto --steps 200 2>>$O/ab.err | sed "s/^/$v /" >> $O/ab.log || exit 1
    done
  done
done
python3 - $O <<'PY'
import json, sys
from collections import defaultdict
O = sys.argv[1]
var = None
for l in open(f"{O}/phases.log"):
    if l.startswith("variant"):
        var = l.split()[1]; continue
    d = json.loads(l)
    for k, v in d["launches"].items():
        if k.startswith("fixup") or k.startswith("sepq60"):
            print(var, k, v["span_us"], v["wave_us"], v["phases_cycles"])
r = defaultdict(list)
for l in open(f"{O}/ab.log"):
    v, j = l.split(" ", 1)
    b = json.loads(j); r[(v, b["width"])].append(b["avg_ms"])
for k in sorted(r): print(k, ["%.5f" % x for x in r[k]])
PY
