#!/bin/bash
# Round-2 GPU call E: PMC + trace of every single-GPU config (D=8 default and D=1), frame series.
set -u
O=gpurun_out/r02e; mkdir -p $O
timeout -k 10 120 python -u tools/frame_series.py > $O/frame_series.log 2>&1 || exit 11
bash tools/gpu/pmc_configs.sh r02e > $O/pmc.log 2>&1 || exit 12
echo done
