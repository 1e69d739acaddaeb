#!/bin/bash
# round 3: PMC + trace of every single-GPU config on the last build of the round (tools/gpu/pmc_configs.sh)
set -o pipefail
bash tools/gpu/pmc_configs.sh r03h c3A c1 c2 c3B c5 c3A_D1 c5_D1 > gpurun_out/pmc_r03h.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_r03h.log; exit 1; }
tail -8 gpurun_out/pmc_r03h.log
