#!/bin/bash
# round 3: bloom chain per-kernel trace + LDS/wait PMC of the current build (XCD block order)
set -o pipefail
O=gpurun_out/r03f; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/bench_bloom.py --steps 100 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-include-regex "up2|yq|final|pass_kernel" --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $O/pmc1 -o run -- python tools/bench_bloom.py --steps 5 --warmup 2 > $O/pmc1.log 2>&1 || { tail -5 $O/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-include-regex "up2|yq|final|pass_kernel" --pmc FETCH_SIZE --output-format csv -d $O/pmc2 -o run -- python tools/bench_bloom.py --steps 5 --warmup 2 > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
PY
for p in pmc1 pmc2; do f=$(find $O/$p -name "*counter_collection.csv" | head -1); python - "$f" <<'PY'
import csv,sys,collections
acc=collections.defaultdict(float); cnt=collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k=(r['Kernel_Name'].split('(')[0][-24:], r['Grid_Size'])
    acc[(k, r['Counter_Name'])]+=float(r['Counter_Value']); cnt[(k, r['Counter_Name'])]+=1
ks=sorted({k for k,_ in acc})
for k in ks:
    g=lambda c: acc[(k,c)]/max(1,cnt[(k,c)])
    if g('SQ_WAVES'):
        print(k, 'conflict/idx', round(g('SQ_LDS_BANK_CONFLICT')/max(1,g('SQ_LDS_IDX_ACTIVE')),3), 'lds/wave', round(g('SQ_INSTS_LDS')/max(1,g('SQ_WAVES')),1),
              'valu/wave', round(g('SQ_INSTS_VALU')/max(1,g('SQ_WAVES')),1), 'wait', round(g('SQ_WAIT_ANY')/max(1,g('SQ_WAVE_CYCLES')),3),
              'busy_cyc', round(g('SQ_BUSY_CYCLES')))
    else:
        print(k, 'FETCH_MB_x2', round(2*g('FETCH_SIZE')/1024,1))
PY
done
