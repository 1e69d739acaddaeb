#!/bin/bash
# round 6: one-frame launches per camera and exact build (tools/probe_camera_tail.py)
set -u -o pipefail
source tools/gpu/outdir.sh r06 camtail
timeout -k 10 300 python -u tools/probe_camera_tail.py "$@" > $O/camtail.log 2>&1 || { tail -30 $O/camtail.log; exit 1; }
cat $O/camtail.log
