#!/bin/bash
# round 3: PMC + trace of every single-GPU config on the final march build (tools/gpu/pmc_configs.sh)
set -o pipefail
bash tools/gpu/pmc_configs.sh r03f c3A c1 c2 c3B c5 c3A_D1 c5_D1 > gpurun_out/pmc_r03f.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_r03f.log; exit 1; }
tail -8 gpurun_out/pmc_r03f.log
