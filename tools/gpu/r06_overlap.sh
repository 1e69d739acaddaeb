#!/bin/bash
# round 6: march + bloom overlap probe (stream priorities, CU masks) at the three frame sizes
set -u -o pipefail
source tools/gpu/outdir.sh r06 overlap
for s in "1920 1080 256" "1280 720 256" "4096 2048 512"; do
  set -- $s
  timeout -k 10 240 python -u tools/probe_overlap.py --width $1 --height $2 --max-iters $3 --frames 64 > $O/ov_$1.log 2>&1 || { tail -30 $O/ov_$1.log; exit 1; }
  tail -1 $O/ov_$1.log
done
