#!/bin/bash
# round 6: the app-frame bench with more hardware queues per process (is queue sharing what slows 2 march streams?)
set -u -o pipefail
source tools/gpu/outdir.sh r06 frameq
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u tools/bench_frame.py --cus "" > $O/frame8.log 2>&1 || { tail -30 $O/frame8.log; exit 1; }
grep width $O/frame8.log
