#!/bin/bash
# PMC passes of the bloom chain's kernels on the final build (one counter group per pass).
set -u
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r02bq; mkdir -p $O
cd /tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
G2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD"
i=0
for G in "$G1" "$G2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-include-regex bloom --pmc $G --output-format csv -d $O/p$i -o run -- python3 $ROOT/tools/bench_bloom.py --steps 10 --warmup 2 > $O/p$i.log 2>&1 || exit $i
done
echo done
