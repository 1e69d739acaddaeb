#!/bin/bash
# GPU suite on the DeviceScope host build, then rocprofv3 kernel trace + 4 PMC passes of every
# single-GPU configuration on the atan2 build.
set -u
mkdir -p gpurun_out/r02am
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02am/pytest_gpu.log 2>&1 || exit 10
timeout -k 10 1500 bash tools/gpu/pmc_configs.sh r02h > gpurun_out/pmc_r02h.log 2>&1 || exit 11
echo done
