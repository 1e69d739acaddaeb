#!/bin/bash
# rocprofv3 kernel trace + 4 PMC passes of every single-GPU configuration on the atan2 build.
set -u
timeout -k 10 1500 bash tools/gpu/pmc_configs.sh r02h > gpurun_out/pmc_r02h.log 2>&1 || exit 11
echo done
