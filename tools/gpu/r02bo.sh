#!/bin/bash
# rocprofv3 kernel trace + stats of the bench command itself (default, and the driver's
# --warmup 5 --steps 20), with the bench line of the same run, for the trace / HIP-event agreement.
set -u
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r02bo; mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/default -o run -- python3 $ROOT/bench.py > $O/default.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/w5 -o run -- python3 $ROOT/bench.py --warmup 5 --steps 20 > $O/w5.log 2>&1 || exit 2
echo done
