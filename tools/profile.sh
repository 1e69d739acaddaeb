#!/bin/bash
# Profile the march kernel with rocprofv3 (run on the GPU box from the repo root):
#   tools/profile.sh TAG [prof_frames.py args...]
#   tools/profile.sh TAG bench [bench.py args...]     (profile the bench command itself)
# Pass 1: kernel trace + stats.  Passes 2-5: PMC counters, one group per pass (never combined with
# tracing domains).  Output: gpurun_out/prof_TAG/{trace,pmc1..pmc4}/...
set -u
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
DRV="python3 $GRAFT_REPO_ROOT/tools/prof_frames.py"
if [ "${1:-}" = "bench" ]; then shift; DRV="python3 $GRAFT_REPO_ROOT/bench.py"; fi
KF="--kernel-include-regex march"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $DRV "$@" > "$OUT/trace.log" 2>&1 || exit 1
grep -h "^{\"metric\"" "$OUT/trace.log" > "$OUT/bench_line.json" || true
timeout -k 10 240 rocprofv3 $KF --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d "$OUT/pmc1" -o run -- $DRV "$@" > "$OUT/pmc1.log" 2>&1 || exit 2
timeout -k 10 240 rocprofv3 $KF --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d "$OUT/pmc2" -o run -- $DRV "$@" > "$OUT/pmc2.log" 2>&1 || exit 3
timeout -k 10 240 rocprofv3 $KF --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc3" -o run -- $DRV "$@" > "$OUT/pmc3.log" 2>&1 || exit 4
timeout -k 10 240 rocprofv3 $KF --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc4" -o run -- $DRV "$@" > "$OUT/pmc4.log" 2>&1 || exit 5
echo "profile $TAG ok"
