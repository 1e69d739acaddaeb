#!/bin/bash
# The app's frame (bh_presenter): presenter parity, the app-frame bench (tools/bench_frame.py) at one frame and 16
# frames per call, and rocprofv3 kernel traces of the default presenter with the march / bloom overlap they show
# (tools/prof_overlap.py):   bash tools/gpu/frame.sh        -> gpurun_out/r06/frame/<time>/
set -u -o pipefail
source tools/gpu/outdir.sh r06 frame
timeout -k 10 600 python -u -m pytest tests/test_gpu_present.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u tools/bench_frame.py > $O/frame.log 2>&1 || { tail -30 $O/frame.log; exit 1; }
grep width $O/frame.log
timeout -k 10 400 python -u tools/bench_frame.py --batch 16 --variants "" --cus "" > $O/frame_b16.log 2>&1 || { tail -30 $O/frame_b16.log; exit 1; }
grep width $O/frame_b16.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for sz in 1920x1080:256 4096x2048:512; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_${sz%%:*} -o run -- python3 tools/bench_frame.py --sizes $sz --only-pipelined --no-roofline > $O/trace_${sz%%:*}.log 2>&1 || { tail -20 $O/trace_${sz%%:*}.log; exit 1; }
  python3 tools/prof_overlap.py $(find $O/trace_${sz%%:*} -name "*kernel_trace.csv" | head -1) | tee $O/overlap_${sz%%:*}.json
done
