#!/bin/bash
# round 3: interleaved march A/B over several libraries (LIBS: "base" = the in-tree build, or variant .so
# paths), REPS rounds of the headline (c3) and config 5 at one frame per launch (c5d1); OUT names the dir
set -o pipefail
O=gpurun_out/${OUT:-r03ab}; mkdir -p $O
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  if [ "$lib" = base ]; then timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  else BH_LIB=$lib timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; fi
  python -c "import json,sys; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_frame'], d['kernel']['ms_per_frame'], d['clock']['mhz'] if d.get('clock') else None)"
}
for r in $(seq 1 ${REPS:-2}); do
  i=0
  for lib in ${LIBS:-base}; do
    i=$((i+1))
    run c3_${i}_$r $lib --steps 20 --warmup 10
    [ -n "$NO_D1" ] || run c5d1_${i}_$r $lib --config 5 --frames-per-launch 1 --steps 100 --warmup 30
  done
done
