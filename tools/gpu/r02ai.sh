#!/bin/bash
set -u
O=gpurun_out/r02ai; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_c_example.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_c_example.log 2>&1 || exit 11
timeout -k 10 120 ./examples/render_frame 4096 2048 512 $O/frame.ppm > $O/render_frame.log 2>&1 || exit 12
echo done
