#!/bin/bash
# The round-6 probes, one per call:
#   bash tools/gpu/probes.sh camtail [probe args]   one-frame launches per camera and exact build (tools/probe_camera_tail.py)
#   bash tools/gpu/probes.sh orbit                  one-frame launches of a moving vs a repeated rotated camera (tools/probe_orbit_single.py)
#   bash tools/gpu/probes.sh rank0                  rank 0's render + unpack at N = 8 with CU-masked unpack shares (tools/probe_rank0.py)
#   bash tools/gpu/probes.sh overlap                march + bloom overlap: stream priorities, CU masks (tools/probe_overlap.py)
# Output: gpurun_out/r06/<probe>/<time>/
set -u -o pipefail
P=${1:?probe}; shift
source tools/gpu/outdir.sh r06 $P
case $P in
  camtail) timeout -k 10 300 python -u tools/probe_camera_tail.py "$@" > $O/camtail.log 2>&1 || { tail -30 $O/camtail.log; exit 1; }
           cat $O/camtail.log ;;
  orbit)   for st in 0 20; do
             timeout -k 10 250 python -u tools/probe_orbit_single.py --start $st > $O/p$st.log 2>&1 || { tail -30 $O/p$st.log; exit 1; }
           done
           grep -h start $O/p*.log ;;
  rank0)   timeout -k 10 500 python -u tools/probe_rank0.py --n 8 --D 64 --root-ratio auto --cu-split 0,16,32,48,64 --it 6 > $O/rank0.jsonl 2>&1 || { tail -30 $O/rank0.jsonl; exit 1; }
           cat $O/rank0.jsonl ;;
  overlap) for s in "1920 1080 256" "1280 720 256" "4096 2048 512"; do
             set -- $s
             timeout -k 10 240 python -u tools/probe_overlap.py --width $1 --height $2 --max-iters $3 --frames 64 > $O/ov_$1.log 2>&1 || { tail -30 $O/ov_$1.log; exit 1; }
             tail -1 $O/ov_$1.log
           done ;;
  *) echo "unknown probe $P" >&2; exit 2 ;;
esac
