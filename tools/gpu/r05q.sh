#!/bin/bash
# round 5: fix-up records (one dependent round trip fewer in fixup_gather_kernel) -- bloom parity, interleaved
# A/B against the list-then-plan form (BH_BLOOM_FIXUP_NOREC=1)
set -u -o pipefail
source tools/gpu/outdir.sh r05 q
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || { tail -30 $O/pytest_bloom.log; exit 1; }
tail -1 $O/pytest_bloom.log
for rep in 1 2 3; do
  for v in rec norec; do
    E=""; if [ $v = norec ]; then E="BH_BLOOM_FIXUP_NOREC=1"; fi
    for s in "1920 1080" "1280 720"; do
      set -- $s
      env $E timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --schedule auto --steps 200 2>>$O/ab.err | sed "s/^/$v /" >> $O/ab.log || exit 1
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
