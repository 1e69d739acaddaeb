#!/bin/bash
# rocprofv3 kernel trace + PMC passes (one counter group per pass, never with tracing domains) of the
# bench, for every BASELINE single-GPU configuration (and the N=8 shard workloads rendered as rank 0
# would: --width/--height and a shard are not bench options, so those use tools/prof_shard.py).
#   bash tools/gpu/pmc_configs.sh TAG [config ...]      -> gpurun_out/pmc_TAG/<config>/...
# then: python tools/pmc_summary.py gpurun_out/pmc_TAG  (writes profiles/pmc_traffic.json entries)
set -u
TAG=$1; shift
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU"
G2="GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_BANK_CONFLICT"
declare -A CFG
CFG[c1]="--width 256 --height 256 --max-iters 64 --surfaces off"
CFG[c2]="--width 1920 --height 1080 --max-iters 256 --camera B"
CFG[c3A]=""
CFG[c3B]="--camera B"
CFG[c5]="--max-iters 1000 --camera C"
CFG[c3A_D1]="--frames-per-launch 1"
CFG[c5_D1]="--max-iters 1000 --camera C --frames-per-launch 1"
# config 1's per-wave fixed cost: the same frame at cap 1 and 2 (VALU per wave = fixed + steps x per-step)
CFG[c1cap1]="--width 256 --height 256 --max-iters 1 --surfaces off"
CFG[c1cap2]="--width 256 --height 256 --max-iters 2 --surfaces off"
LIST="${@:-c1 c2 c3A c3B c5 c3A_D1 c5_D1}"
for C in $LIST; do
  OUT=$ROOT/gpurun_out/pmc_$TAG/$C
  mkdir -p $OUT
  # a step is one batch (one launch); one-frame launches get more of them
  case $C in *_D1) SW="--steps 100 --warmup 30";; *) SW="--steps 20 --warmup 10";; esac
  A="$ROOT/bench.py --no-cpu --no-extra $SW ${CFG[$C]}"
  echo "$A" > $OUT/cmd.txt
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $A > $OUT/trace.log 2>&1 || exit 1
  i=0
  for G in "$G1" "$G2" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-include-regex march_tile --pmc $G --output-format csv -d $OUT/p$i -o run -- python3 $A > $OUT/p$i.log 2>&1 || exit $((i+1))
  done
  echo "$C ok"
done
