#!/bin/bash
set -u
O=gpurun_out/r02u; mkdir -p $O
timeout -k 10 300 python -u tools/orbit_probe.py --angles 0,0.2,0.4,1,5,20 > $O/orbit_probe.log 2>&1 || exit 11
echo done
