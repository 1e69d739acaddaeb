#!/bin/bash
# bloom PMC at a frame size: where each kernel's wave cycles go (parked on waits, issue stalls, active),
# instructions per wave, LDS bank conflicts.   OUT=tag tools/gpu/bloom_pmc.sh W H
set -o pipefail
W=${1:-1920}; H=${2:-1080}
export O=gpurun_out/${OUT:-bloom_pmc_$W}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM"
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $O/p1 -o run -- python tools/bench_bloom.py --width $W --height $H --steps 10 --warmup 2 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $O/p2 -o run -- python tools/bench_bloom.py --width $W --height $H --steps 10 --warmup 2 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
python tools/bloom_pmc_summary.py $O > $O/summary.txt
