#!/bin/bash
# round 3: bloom -- exact fma forms and compile-time standard plans and
# the footprint loads issued before the table loads; GPU suite, then interleaved chain A/B vs HEAD's build
set -o pipefail
export O=gpurun_out/${OUT:-r03h}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
b() {  # name [lib] [env]
  local n=$1
  if [ -n "$2" ]; then env BH_LIB=$2 $3 timeout -k 10 120 python tools/bench_bloom.py --steps 200 > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  else env $3 timeout -k 10 120 python tools/bench_bloom.py --steps 200 > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; fi
  python -c "import json; d=[json.loads(l) for l in open('$O/$n.json') if l.startswith('{')]; print('$n', *[(x['bloom_schedule'], x['avg_ms'], x['min_ms']) for x in d])"
}
for r in 1 2 3; do
  b new_$r
  b head_$r ${HEADLIB:-tools/variants/head.so}
  b alt_$r "" ${ALT:-BH_BLOOM_NO_STD=1}
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o run -- python tools/bench_bloom.py --steps 100 > $O/prof_new.log 2>&1 || exit 1
python - <<'PY'
import csv, glob, os
for f in glob.glob(os.environ['O'] + '/prof_new/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'bloom' in r['Name'] or 'up2' in r['Name'] or 'pass_kernel' in r['Name']:
            print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us')
PY
