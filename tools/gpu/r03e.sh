#!/bin/bash
# round 3: bloom code-table encoder (BH_BLOOM_ETAB) -- exhaustive self-test, bloom parity of the variant,
# A/B chain time, per-kernel trace and LDS PMC of both builds
set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_crmath.py -k "code_table" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_op10.log 2>&1 || { tail -20 $O/pytest_op10.log; exit 1; }
tail -1 $O/pytest_op10.log
BH_LIB=tools/variants/bloom_etab.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bloom.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_bloom_etab.log 2>&1 || { tail -20 $O/pytest_bloom_etab.log; exit 1; }
tail -1 $O/pytest_bloom_etab.log
for r in 1 2 3; do
  timeout -k 10 120 python tools/bench_bloom.py --steps 300 > $O/base_$r.json 2>$O/base_$r.err || exit 1
  BH_LIB=tools/variants/bloom_etab.so timeout -k 10 120 python tools/bench_bloom.py --steps 300 > $O/etab_$r.json 2>$O/etab_$r.err || exit 1
  grep auto $O/base_$r.json | cut -c1-110; grep auto $O/etab_$r.json | cut -c1-110
done
for v in base etab; do
  L=""; [ $v = etab ] && L=tools/variants/bloom_etab.so
  BH_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python tools/bench_bloom.py --steps 100 > $O/prof_$v.log 2>&1 || exit 1
  BH_LIB=$L timeout -s KILL 90 rocprofv3 --kernel-include-regex "up2|yq|final" --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $O/pmc_$v -o run -- python tools/bench_bloom.py --steps 5 --warmup 2 > $O/pmc_$v.log 2>&1 || exit 1
done
for v in base etab; do echo "== $v"; f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1); python - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'bloom' in r['Name'] or 'up2' in r['Name'] or 'pass_kernel' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
PY
f=$(find $O/pmc_$v -name "*counter_collection.csv" | head -1); python - "$f" <<'PY'
import csv,sys,collections
acc=collections.defaultdict(float); cnt=collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k=(r['Kernel_Name'].split('(')[0][-22:], r['Grid_Size'])
    acc[(k, r['Counter_Name'])]+=float(r['Counter_Value']); cnt[(k, r['Counter_Name'])]+=1
ks=sorted({k for k,_ in acc})
for k in ks:
    g=lambda c: acc[(k,c)]/max(1,cnt[(k,c)])
    print(k, 'conflict/idx', round(g('SQ_LDS_BANK_CONFLICT')/max(1,g('SQ_LDS_IDX_ACTIVE')),3), 'lds/wave', round(g('SQ_INSTS_LDS')/max(1,g('SQ_WAVES')),1),
          'valu/wave', round(g('SQ_INSTS_VALU')/max(1,g('SQ_WAVES')),1), 'wait', round(g('SQ_WAIT_ANY')/max(1,g('SQ_WAVE_CYCLES')),3))
PY
done
