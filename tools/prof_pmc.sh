#!/bin/bash
# PMC passes (one counter group per pass, no tracing) over any python command, kernels matching REGEX:
#   tools/prof_pmc.sh TAG REGEX script.py [args...]   -> gpurun_out/pmc_TAG/{p1..p3}/
set -u
TAG=$1; RE=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
S=$GRAFT_REPO_ROOT/$1; shift
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS"
G2="GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_ACTIVE_INST_LDS"
i=0
for G in "$G1" "$G2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-include-regex "$RE" --pmc $G --output-format csv -d "$OUT/p$i" -o run -- python3 $S "$@" > "$OUT/p$i.log" 2>&1 || exit $i
done
echo "pmc $TAG ok"
