#!/bin/bash
# round 6: stream priority / march-stream variants of the march + bloom overlap (after the tail fix)
set -u -o pipefail
source tools/gpu/outdir.sh r06 overlap3
V=normal,bloom_high,bloom_low,march_high,2march_normal,2march_bloom_high,2march_bloom_low,2march_march_high
for s in "1920 1080 256" "1280 720 256" "4096 2048 512"; do
  set -- $s
  timeout -k 10 240 python -u tools/probe_overlap.py --width $1 --height $2 --max-iters $3 --frames 64 --variants $V > $O/ov_$1.log 2>&1 || { tail -30 $O/ov_$1.log; exit 1; }
  tail -1 $O/ov_$1.log
done
