#!/bin/bash
# Config 1 on the no-surface instantiation at 256 frames per launch: bench with the oracle leg, then the
# rocprofv3 trace + PMC passes (pmc_traffic.json key _D256).
set -u
mkdir -p gpurun_out/r02ay
timeout -k 10 300 python -u bench.py --config 1 > gpurun_out/r02ay/c1_256x256_cap64_nosurf.log 2>&1 || exit 10
timeout -k 10 1200 bash tools/gpu/pmc_configs.sh r02ay c1 > gpurun_out/r02ay/pmc.log 2>&1 || exit 11
echo done
