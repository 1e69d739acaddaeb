#!/bin/bash
# round 6: the app-frame bench with several frames per presenter call (offline camera paths)
set -u -o pipefail
source tools/gpu/outdir.sh r06 frameb
for b in 4 16; do
  timeout -k 10 400 python -u tools/bench_frame.py --cus "" --batch $b --variants d3m1 > $O/frame_b$b.log 2>&1 || { tail -30 $O/frame_b$b.log; exit 1; }
  grep width $O/frame_b$b.log
done
