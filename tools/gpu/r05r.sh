#!/bin/bash
# round 5: the bloom chain's per-kernel roofline inputs (trace + PMC) on the final build, 1920x1080, 1280x720
# and 4096x2048
set -u -o pipefail
source tools/gpu/outdir.sh r05 r
for s in "1920 1080" "1280 720" "4096 2048"; do
  set -- $s
  tools/gpu/bloom_roofline.sh $1 $2 $O/roof$1 || exit 1
done
echo done
