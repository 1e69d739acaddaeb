#!/bin/bash
# round 3: (1) sky staged in LDS (north_star) A/B: parity of the variant on the full-frame config tests,
# interleaved bench A/B; (2) bloom XCD-order A/B with per-kernel times; (3) N>1 rehearsals.
set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
BH_LIB=tools/variants/sky_lds.so timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_random.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_skylds.log 2>&1 || { echo "sky_lds parity failed"; tail -30 $O/pytest_skylds.log; exit 1; }
tail -1 $O/pytest_skylds.log
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  if [ "$lib" = base ]; then timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  else BH_LIB=$lib timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; fi
  python -c "import json,sys; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_frame'], d['kernel']['ms_per_frame'], d['clock']['mhz'] if d.get('clock') else None)"
}
for r in 1 2; do
  run c3_base_$r base --steps 20 --warmup 10
  run c3_skylds_$r tools/variants/sky_lds.so --steps 20 --warmup 10
  run c5_base_$r base --config 5 --steps 20 --warmup 10
  run c5_skylds_$r tools/variants/sky_lds.so --config 5 --steps 20 --warmup 10
  run c2_base_$r base --config 2 --steps 20 --warmup 10
  run c2_skylds_$r tools/variants/sky_lds.so --config 2 --steps 20 --warmup 10
done
for r in 1 2; do
  timeout -k 10 120 python tools/bench_bloom.py --steps 200 > $O/bloom_xcd_$r.json 2>$O/bloom_xcd_$r.err || exit 1
  BH_LIB=tools/variants/bloom_noxcd.so timeout -k 10 120 python tools/bench_bloom.py --steps 200 > $O/bloom_noxcd_$r.json 2>$O/bloom_noxcd_$r.err || exit 1
  grep auto $O/bloom_xcd_$r.json | cut -c1-120; grep auto $O/bloom_noxcd_$r.json | cut -c1-120
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
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --verify-gather > $O/reh2.json 2> $O/reh2.err || { tail -20 $O/reh2.err; exit 1; }
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 3 --steps 10 --warmup 3 --verify-gather --fmt bgra8 > $O/reh3.json 2> $O/reh3.err || { tail -20 $O/reh3.err; exit 1; }
python - <<'PY'
import json
for f in ("reh2", "reh3"):
    d = json.loads(open(f"gpurun_out/r03d/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("gather_verified_bit_exact"), json.dumps(d.get("ranks")))
PY
