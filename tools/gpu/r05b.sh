#!/bin/bash
# round 5: the quad separable up pass's wave phases (tools/probe_bloom_phases.py) at 1920x1080 and 1280x720,
# and the bloom chain's per-kernel roofline inputs (trace + PMC) at 1920x1080 and 4096x2048
set -u
source tools/gpu/outdir.sh r05 b
for s in "1920 1080" "1280 720"; do
  set -- $s
  BH_LIB=tools/variants/bphase.so timeout -k 10 120 python tools/probe_bloom_phases.py --width $1 --height $2 >> $O/phases.log 2>&1 || exit 1
done
for s in "1920 1080" "4096 2048"; do
  set -- $s
  tools/gpu/bloom_roofline.sh $1 $2 $O/roof$1 || exit 1
done
