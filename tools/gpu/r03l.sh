#!/bin/bash
# round 3: final-build profiles -- rocprofv3 kernel trace + PMC passes of every single-GPU config under
# the step = batch protocol (tools/gpu/pmc_configs.sh), and the driver's bench command traced
set -o pipefail
O=gpurun_out/r03l; mkdir -p $O
bash tools/gpu/pmc_configs.sh r03 c3A c1 c2 c3B c5 c3A_D1 c5_D1 > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
tail -8 $O/pmc.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/driver_cmd -o run -- python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err || { echo "driver cmd failed"; tail -5 $O/driver_cmd.err; exit 1; }
tail -c 600 $O/driver_cmd.json
