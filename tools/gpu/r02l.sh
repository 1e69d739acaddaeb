#!/bin/bash
set -u
O=gpurun_out/r02l; mkdir -p $O
timeout -k 10 200 python -u tools/clock_series.py > $O/clock_series.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/probe_rank0.py --n 8 --rows 32,64,128 --frame 8192x4096 > $O/rank0_config4.log 2>&1 || exit 14
echo done
