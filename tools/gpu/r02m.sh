#!/bin/bash
set -u
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 200 python -u tools/clock_series.py --frames 50 > $O/clock_series.log 2>&1 || exit 11
echo done
