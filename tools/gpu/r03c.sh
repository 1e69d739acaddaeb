#!/bin/bash
# round 3: bloom chain A/B -- XCD-aware block order vs the raw grid order; per-kernel times (rocprofv3)
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  timeout -k 10 120 python tools/bench_bloom.py --steps 200 > $O/xcd_$r.json 2>$O/xcd_$r.err || exit 1
  BH_LIB=tools/variants/bloom_noxcd.so timeout -k 10 120 python tools/bench_bloom.py --steps 200 > $O/noxcd_$r.json 2>$O/noxcd_$r.err || exit 1
  grep auto $O/xcd_$r.json; grep auto $O/noxcd_$r.json
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_xcd -o run -- python tools/bench_bloom.py --steps 100 > $O/prof_xcd.log 2>&1 || exit 1
BH_LIB=tools/variants/bloom_noxcd.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_noxcd -o run -- python tools/bench_bloom.py --steps 100 > $O/prof_noxcd.log 2>&1 || exit 1
for v in xcd noxcd; do echo "== $v"; f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1); python - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'bloom' in r['Name'] or 'up2' in r['Name'] or 'pass_kernel' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
PY
done
# N>1 rehearsals (all ranks on cuda:0 over gloo): the per-rank breakdown and the gather check of the last batch
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --verify-gather > $O/reh2.json 2> $O/reh2.err || { tail -20 $O/reh2.err; exit 1; }
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 3 --steps 10 --warmup 3 --verify-gather --fmt bgra8 > $O/reh3.json 2> $O/reh3.err || { tail -20 $O/reh3.err; exit 1; }
python - <<'PY'
import json
for f in ("reh2", "reh3"):
    d = json.loads(open(f"gpurun_out/r03c/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("gather_verified_bit_exact"), json.dumps(d.get("ranks")))
PY
