#!/bin/bash
# round 5: the final epilogue's in-block fix (FIX2) -- bloom parity, then interleaved A/B of the chain:
# both fixes (default), the Y fix only (BH_BLOOM_NO_FIX=2), neither (=1)
set -u -o pipefail
source tools/gpu/outdir.sh r05 i
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || { tail -30 $O/pytest_bloom.log; exit 1; }
tail -1 $O/pytest_bloom.log
for rep in 1 2 3; do
  for v in 0 2 1; do
    for s in "1920 1080" "1280 720"; do
      set -- $s
      BH_BLOOM_NO_FIX=$v timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --schedule auto --steps 200 2>>$O/ab.err | sed "s/^/nofix$v /" >> $O/ab.log || exit 1
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
