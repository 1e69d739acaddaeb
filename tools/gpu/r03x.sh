#!/bin/bash
# round 3: where a 1920x1080 bloom frame goes (literal schedule): kernel trace per pass, grid and time
set -o pipefail
export O=gpurun_out/${OUT:-r03x}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python tools/bench_bloom.py --steps 20 --warmup 5 --width ${W:-1920} --height ${H:-1080} > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python - <<'PY'
import csv, glob, collections, os
rows = []
for f in glob.glob(os.environ["O"] + "/trace/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(list)
for r in rows:
    k = (r['Kernel_Name'][:60], r.get('Grid_Size_X', r.get('Grid_Size', '')), r.get('Grid_Size_Y', ''))
    agg[k].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
tot = 0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    print('%-60s grid %s x %s  n=%4d avg %.2f us  sum %.0f us' % (k[0], k[1], k[2], len(v), sum(v) / len(v), sum(v)))
print('total us', round(tot))
PY
