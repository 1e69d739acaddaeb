#!/bin/bash
# round 6: the GPU test suite (optionally a -k expression), the app-frame bench, the camera tail probe
set -u -o pipefail
source tools/gpu/outdir.sh r06 suite
K=${1:-}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u tools/bench_frame.py > $O/frame.log 2>&1 || { tail -30 $O/frame.log; exit 1; }
grep width $O/frame.log
for cap in 128 512; do
  timeout -k 10 200 python -u tools/probe_camera_tail.py --cameras A,B --max-iters $cap --reps 8 >> $O/camtail.log 2>&1 || { tail -30 $O/camtail.log; exit 1; }
done
grep camera $O/camtail.log
