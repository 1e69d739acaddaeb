#!/bin/bash
# Shader clock per frame after idle / hot; rank 0 render + unpack sweep (rows in flight) with the
# all-loads-in-flight unpack staging; unpack parity tests.
set -u
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 200 python -u tools/clock_series.py > $O/clock_series.log 2>&1 || exit 11
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -k "unpack or rgbm or shard" --timeout 120 --timeout-method thread > $O/pytest_unpack.log 2>&1 || exit 12
timeout -k 10 400 python -u tools/probe_rank0.py --n 2,4,8 --rows 16,64,0 --frame 4096x2048 > $O/rank0_strong.log 2>&1 || exit 13
timeout -k 10 300 python -u tools/probe_rank0.py --n 8 --rows 16,0 --frame 8192x4096 > $O/rank0_config4.log 2>&1 || exit 14
echo done
