#!/bin/bash
set -u
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 200 python -u tools/heavy_clock.py > $O/heavy_clock.log 2>&1 || exit 11
echo done
