#!/bin/bash
# round 5: per-wave timelines of the quad passes and the fix-up after the column strips and the late own loads
set -u -o pipefail
source tools/gpu/outdir.sh r05 phases_late
for s in "1920 1080" "1280 720"; do
  set -- $s
  BH_LIB=tools/variants/bphase.so timeout -k 10 120 python tools/probe_bloom_phases.py --width $1 --height $2 --chains 5 >> $O/phases.log 2>> $O/phases.err || { tail -20 $O/phases.err; exit 1; }
done
python3 - $O/phases.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    for k, v in d["launches"].items():
        print(d["width"], k, v["span_us"], v["wave_us"], v["ramp_us"], v["tail_us"], v["mean_resident"], v["phases_share"])
PY
