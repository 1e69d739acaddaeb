#!/bin/bash
# round 5: blocks-per-CU caps of the quad passes (BH_BLOOM_CAP_*: 2 full rounds of resident waves instead of
# 1.33) -- interleaved A/B of the chain at 1920x1080 and 1280x720, parity of the best
set -u -o pipefail
source tools/gpu/outdir.sh r05 l
for rep in 1 2 3; do
  for v in base f4 f5 p4 p4f4; do
    E=""
    case $v in f4) E="BH_BLOOM_CAP_FINAL=4";; f5) E="BH_BLOOM_CAP_FINAL=5";; p4) E="BH_BLOOM_CAP_PLAIN=4";; p4f4) E="BH_BLOOM_CAP_PLAIN=4 BH_BLOOM_CAP_FINAL=4";; esac
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
