#!/bin/bash
# round 3: fixed per-wave cost -- host reciprocals for vs_main's interpolation, the sky gathers issued
# together, atan2's f64 coefficients as SGPR operands -- GPU suite, then interleaved A/B vs HEAD's build
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  if [ "$lib" = base ]; then timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  else BH_LIB=$lib timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; fi
  python -c "import json,sys; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_frame'], d['kernel']['ms_per_frame'], d['clock']['mhz'] if d.get('clock') else None)"
}
for r in 1 2 3; do
  run c3_new_$r base --steps 20 --warmup 10
  run c3_head_$r tools/variants/head.so --steps 20 --warmup 10
  run c1_new_$r base --config 1 --steps 10 --warmup 5
  run c1_head_$r tools/variants/head.so --config 1 --steps 10 --warmup 5
done
for r in 1 2; do
  run c2_new_$r base --config 2 --steps 20 --warmup 10
  run c2_head_$r tools/variants/head.so --config 2 --steps 20 --warmup 10
  run c5d1_new_$r base --config 5 --frames-per-launch 1 --steps 100 --warmup 30
  run c5d1_head_$r tools/variants/head.so --config 5 --frames-per-launch 1 --steps 100 --warmup 30
done
