#!/bin/bash
# round 6: why is a one-frame march launch with a moving camera slow? cameras A / B / orbit, host enqueue time,
# and a kernel trace of the orbit run at 4096x2048
set -u -o pipefail
source tools/gpu/outdir.sh r06 overlap2
for cam in A B orbit; do
  timeout -k 10 120 python -u tools/probe_overlap.py --width 4096 --height 2048 --max-iters 512 --frames 32 --camera $cam --only-march >> $O/cams.log 2>&1 || { tail -30 $O/cams.log; exit 1; }
done
cat $O/cams.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/probe_overlap.py --width 4096 --height 2048 --max-iters 512 --frames 32 --camera orbit --variants normal > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
tail -1 $O/prof.log
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
