#!/bin/bash
# round 3: march A/B -- the working tree against OLDLIB (a variant .so), interleaved, after the GPU suite
# (OUT names the output directory)
set -o pipefail
O=gpurun_out/${OUT:-r03r}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  if [ "$lib" = base ]; then timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  else BH_LIB=$lib timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; fi
  python -c "import json,sys; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_frame'], d['kernel']['ms_per_frame'], d['clock']['mhz'] if d.get('clock') else None)"
}
for r in 1 2 3; do
  run c5d1_new_$r base --config 5 --frames-per-launch 1 --steps 100 --warmup 30
  run c5d1_old_$r ${OLDLIB:-tools/variants/noeprio.so} --config 5 --frames-per-launch 1 --steps 100 --warmup 30
  run c3_new_$r base --steps 20 --warmup 10
  run c3_old_$r ${OLDLIB:-tools/variants/noeprio.so} --steps 20 --warmup 10
done
for r in 1 2; do
  run c3d1_new_$r base --frames-per-launch 1 --steps 100 --warmup 30
  run c3d1_old_$r ${OLDLIB:-tools/variants/noeprio.so} --frames-per-launch 1 --steps 100 --warmup 30
  run c5_new_$r base --config 5 --steps 20 --warmup 10
  run c5_old_$r ${OLDLIB:-tools/variants/noeprio.so} --config 5 --steps 20 --warmup 10
  run c2_new_$r base --config 2 --steps 20 --warmup 10
  run c2_old_$r ${OLDLIB:-tools/variants/noeprio.so} --config 2 --steps 20 --warmup 10
  run c1_new_$r base --config 1 --steps 20 --warmup 10
  run c1_old_$r ${OLDLIB:-tools/variants/noeprio.so} --config 1 --steps 20 --warmup 10
done
