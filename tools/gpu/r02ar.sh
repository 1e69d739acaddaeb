#!/bin/bash
# Every single-GPU config with its CPU leg (parity + cpu_baseline) on the prepared-launch build.
set -u
timeout -k 10 900 bash tools/configs.sh > gpurun_out/configs_r02ar.log 2>&1 || exit 11
echo done
