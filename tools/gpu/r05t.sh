#!/bin/bash
# round 5: per-wave timelines of the quad passes and the fix-up pass (diagnostic build, BH_BLOOM_PHASES);
# BH_BLOOM_PHASES_FIXUP_PART 1 / 2: the fix-up's rows / columns alone (timing only)
set -u -o pipefail
source tools/gpu/outdir.sh r05 fixup_phases
for part in 0 1 2; do
  for s in "1920 1080" "1280 720"; do
    set -- $s
    echo "part $part" >> $O/phases.log
    BH_BLOOM_PHASES_FIXUP_PART=$part BH_LIB=tools/variants/bphase.so timeout -k 10 120 python tools/probe_bloom_phases.py --width $1 --height $2 --chains 5 >> $O/phases.log 2>> $O/phases.err || { tail -20 $O/phases.err; exit 1; }
  done
done
python3 - $O/phases.log <<'PY'
import json, sys
part = None
for l in open(sys.argv[1]):
    if l.startswith("part"):
        part = l.split()[1]; continue
    d = json.loads(l)
    for k, v in d["launches"].items():
        if k.startswith("fixup"):
            print(part, d["width"], k, v["span_us"], v["wave_us"], v["waves"], v["phases_cycles"])
PY
