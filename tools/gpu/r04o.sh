#!/bin/bash
# round 4: why a shard's tiles cost more than the one-GPU frame's -- the march kernel's counters per wave
# for n = 1 (packed layout) and n = 8 (shard 1), 16 frames per launch
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r04o; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
P2="FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVES"
for n in 1 8; do
  A="$GRAFT_REPO_ROOT/tools/probe_rank0.py --n $n --D 16 --rows 64 --root-ratio 1 --transport rgbm14 --it 4"
  i=0
  for G in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --kernel-include-regex march_tile --pmc $G --output-format csv -d $O/n${n}_p$i -o run -- python3 $A > $O/n${n}_p$i.log 2>&1 || exit 1
  done
done
