#!/bin/bash
# round 3: the two-op x/6 and x/12 cores -- the GPU suite (selftest ops 1 and 5 are exhaustive over all
# 2^32 patterns), then the working tree against OLDLIB (HEAD before the change), interleaved, on the
# march configs and the bloom chain
set -o pipefail
O=gpurun_out/${OUT:-r03s}; mkdir -p $O
OLD=${OLDLIB:-tools/variants/old.so}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  if [ "$lib" = base ]; then timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  else BH_LIB=$lib timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; fi
  python -c "import json,sys; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_frame'], d['kernel']['ms_per_frame'], d['clock']['mhz'] if d.get('clock') else None)"
}
bloom() {  # name lib
  local n=$1 lib=$2
  if [ "$lib" = base ]; then timeout -k 10 120 python tools/bench_bloom.py --steps 200 > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  else BH_LIB=$lib timeout -k 10 120 python tools/bench_bloom.py --steps 200 > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; fi
  python -c "import json; [print('$n', x['bloom_schedule'], x['avg_ms']) for x in (json.loads(l) for l in open('$O/$n.json') if l.startswith('{'))]"
}
for r in 1 2 3; do
  run c3_new_$r base --steps 20 --warmup 10
  run c3_old_$r $OLD --steps 20 --warmup 10
  run c1_new_$r base --config 1 --steps 20 --warmup 10
  run c1_old_$r $OLD --config 1 --steps 20 --warmup 10
done
for r in 1 2; do
  run c5d1_new_$r base --config 5 --frames-per-launch 1 --steps 100 --warmup 30
  run c5d1_old_$r $OLD --config 5 --frames-per-launch 1 --steps 100 --warmup 30
  run c2_new_$r base --config 2 --steps 20 --warmup 10
  run c2_old_$r $OLD --config 2 --steps 20 --warmup 10
  bloom bloom_new_$r base
  bloom bloom_old_$r $OLD
done
