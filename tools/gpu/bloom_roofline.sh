#!/bin/bash
# The bloom chain's per-kernel roofline inputs at one frame size (tools/bloom_roofline.py --pmc DIR): the
# kernel trace and three PMC passes of tools/bench_bloom.py (fused schedule), each its own rocprofv3 run.
#   tools/gpu/bloom_roofline.sh W H OUTDIR
set -u -o pipefail
W=$1; H=$2; D=$3; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python tools/bench_bloom.py --width $W --height $H --steps 20 --warmup 3 --schedule auto"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $B > $D/trace.log 2>&1 || exit 1
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $D/p1 -o run -- $B > $D/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/p2 -o run -- $B > $D/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/p3 -o run -- $B > $D/p3.log 2>&1 || exit 1
