#!/bin/bash
# round 3: bloom PMC -- where the kernels' wave cycles go (parked on waits, issue stalls, active)
set -o pipefail
export O=gpurun_out/${OUT:-r03i}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM"
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $O/p1 -o run -- python tools/bench_bloom.py --steps 10 --warmup 2 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $O/p2 -o run -- python tools/bench_bloom.py --steps 10 --warmup 2 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
python - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(list)
for f in glob.glob(os.environ["O"] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[(r['Kernel_Name'][:34], r['Counter_Name'])].append(float(r['Counter_Value']))
ks = sorted({k for k, _ in agg})
for k in ks:
    d = {c: sum(v) / len(v) for (kk, c), v in agg.items() if kk == k}
    w = d.get('SQ_WAVES', 0) or 1
    wc = d.get('SQ_WAVE_CYCLES', 0) or 1
    print(k, 'waves', int(w), 'valu/w %.0f lds/w %.0f salu/w %.0f' % (d.get('SQ_INSTS_VALU', 0) / w, d.get('SQ_INSTS_LDS', 0) / w, d.get('SQ_INSTS_SALU', 0) / w),
          'wait %.2f issue-stall %.2f (lds %.2f) active %.2f valu-active %.2f' % (d.get('SQ_WAIT_ANY', 0) / wc, d.get('SQ_WAIT_INST_ANY', 0) / wc, d.get('SQ_WAIT_INST_LDS', 0) / wc, d.get('SQ_ACTIVE_INST_ANY', 0) / wc, d.get('SQ_ACTIVE_INST_VALU', 0) / wc),
          'bankconf/ldsactive %.2f' % (d.get('SQ_LDS_BANK_CONFLICT', 0) / (d.get('SQ_LDS_IDX_ACTIVE', 0) or 1)),
          'wavecyc/wave %.0f' % (wc / w))
PY
