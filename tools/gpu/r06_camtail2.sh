#!/bin/bash
# round 6: one-frame launch time vs the cap, cameras A and B (tools/probe_camera_tail.py)
set -u -o pipefail
source tools/gpu/outdir.sh r06 camtail2
for cap in 64 128 256 512 1000; do
  timeout -k 10 200 python -u tools/probe_camera_tail.py --cameras A,B --max-iters $cap --reps 8 >> $O/camtail.log 2>&1 || { tail -30 $O/camtail.log; exit 1; }
done
grep camera $O/camtail.log
