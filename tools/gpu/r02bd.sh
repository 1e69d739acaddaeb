#!/bin/bash
# PMC passes of the bloom chain (fused + literal) on the TapPlan build.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r02bd; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="$GRAFT_REPO_ROOT/tools/bench_bloom.py --steps 10 --warmup 2"
timeout -s KILL 120 rocprofv3 --kernel-include-regex bloom --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/p1 -o run -- python3 $A > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-include-regex bloom --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $O/p2 -o run -- python3 $A > $O/p2.log 2>&1 || exit 2
echo done
