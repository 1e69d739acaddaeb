#!/bin/bash
# round 3: A/B of library variants (tools/variants/NAME.so) against the working tree, interleaved:
#   VARIANTS="a b" [ROUNDS=2] [CONFIGS="c3 c1 c5d1 c2"] bash tools/gpu/r03u.sh
# First the full-frame parity tests of every config on each variant (tests/test_gpu_configs.py).
set -o pipefail
O=gpurun_out/${OUT:-r03u}; mkdir -p $O
for v in $VARIANTS; do
  BH_LIB=tools/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
declare -A CFG
CFG[c3]="--steps 20 --warmup 10"
CFG[c1]="--config 1 --steps 20 --warmup 10"
CFG[c2]="--config 2 --steps 20 --warmup 10"
CFG[c5]="--config 5 --steps 20 --warmup 10"
CFG[c5d1]="--config 5 --frames-per-launch 1 --steps 100 --warmup 30"
CFG[c3d1]="--frames-per-launch 1 --steps 100 --warmup 30"
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  if [ "$lib" = base ]; then timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  else BH_LIB=tools/variants/$lib.so timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; fi
  python -c "import json,sys; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_frame'], d['kernel']['ms_per_frame'], d['clock']['mhz'] if d.get('clock') else None)"
}
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CONFIGS:-c3 c1 c5d1 c2}; do
    for v in base $VARIANTS; do
      run ${c}_${v}_$r $v ${CFG[$c]} || exit 1
    done
  done
done
