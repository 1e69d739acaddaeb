#!/bin/bash
# round 5: 2- and 3-rank rehearsals of the N>1 path on the current build (all ranks on cuda:0, gather
# verified bit-exact), the bloom grid-origin policy A/B (BH_BLOOM_ORG_GROW), and the rocprofv3 kernel trace
# of the driver's bench command (the profile the bench line's kernel average must agree with)
set -u
source tools/gpu/outdir.sh r05 h
BH_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --verify-gather --steps 4 --warmup 2 --no-cpu > $O/reh2.json 2> $O/reh2.err || { tail -20 $O/reh2.err; exit 1; }
BH_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 3 --verify-gather --steps 4 --warmup 2 --no-cpu > $O/reh3.json 2> $O/reh3.err || { tail -20 $O/reh3.err; exit 1; }
for rep in 1 2 3; do
  for v in keep grow; do
    E=""; if [ $v = grow ]; then E="BH_BLOOM_ORG_GROW=1"; fi
    env $E timeout -k 10 120 python tools/bench_bloom.py --width 1920 --height 1080 --schedule auto --steps 200 2>/dev/null | sed "s/^/$v /" >> $O/ab_org.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_traced.json 2> $O/bench_traced.err || exit 1
python3 - $O <<'PY'
import json, sys, collections
O = sys.argv[1]
for f in ("reh2.json", "reh3.json", "bench_traced.json"):
    j = json.loads([l for l in open(f"{O}/{f}") if l.startswith("{")][-1])
    print(f, j["n_gpus"], j["ms_per_frame"], j.get("gather_verified_bit_exact"), j.get("kernel", {}).get("avg_ms"))
d = collections.defaultdict(list)
for l in open(f"{O}/ab_org.log"):
    v, j = l.split(" ", 1); d[v].append(json.loads(j)["avg_ms"])
for k, x in d.items(): print("org", k, x, sum(x) / len(x))
import csv
for r in csv.DictReader(open(f"{O}/trace/run_kernel_stats.csv")):
    print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
