#!/bin/bash
# round 3: PMC + trace of every single-GPU config on the build with the two-op x/6 and the camera-outside
# step (tools/gpu/pmc_configs.sh), then the summary table
set -o pipefail
bash tools/gpu/pmc_configs.sh r03g c3A c1 c2 c3B c5 c3A_D1 c5_D1 > gpurun_out/pmc_r03g.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_r03g.log; exit 1; }
tail -8 gpurun_out/pmc_r03g.log
