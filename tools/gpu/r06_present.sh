#!/bin/bash
# round 6: presenter parity and the batched app-frame bench
set -u -o pipefail
source tools/gpu/outdir.sh r06 present
timeout -k 10 600 python -u -m pytest tests/test_gpu_present.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for b in 4 16; do
timeout -k 10 400 python -u tools/bench_frame.py --batch $b --variants "" --cus "" --no-roofline > $O/frame_b$b.log 2>&1 || { tail -30 $O/frame_b$b.log; exit 1; }
grep width $O/frame_b$b.log
done
