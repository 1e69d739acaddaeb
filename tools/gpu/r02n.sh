#!/bin/bash
set -u
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 300 python -u tools/ramp_probe.py > $O/ramp.log 2>&1 || exit 11
echo done
