#!/bin/bash
# round 3: the lane-spread tail -- GPU suite, then interleaved A/B against the one-lane-per-ray tail
# (tools/variants/scalar_tail.so) on the tail-bound cases (one frame per launch) and the headline.
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  if [ "$lib" = base ]; then timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  else BH_LIB=$lib timeout -k 10 120 python bench.py --no-cpu --no-extra "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; fi
  python -c "import json,sys; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_frame'], d['kernel']['ms_per_frame'], d['kernel']['name'], d['clock']['mhz'] if d.get('clock') else None)"
}
for r in 1 2; do
  run c5d1_spread_$r base --config 5 --frames-per-launch 1 --steps 100 --warmup 30
  run c5d1_scalar_$r tools/variants/scalar_tail.so --config 5 --frames-per-launch 1 --steps 100 --warmup 30
  run c3d1_spread_$r base --frames-per-launch 1 --steps 100 --warmup 30
  run c3d1_scalar_$r tools/variants/scalar_tail.so --frames-per-launch 1 --steps 100 --warmup 30
  run c2d1_spread_$r base --config 2 --frames-per-launch 1 --steps 100 --warmup 30
  run c2d1_scalar_$r tools/variants/scalar_tail.so --config 2 --frames-per-launch 1 --steps 100 --warmup 30
  run c3_spread_$r base --steps 20 --warmup 10
  run c3_scalar_$r tools/variants/scalar_tail.so --steps 20 --warmup 10
  run c5_spread_$r base --config 5 --steps 20 --warmup 10
  run c5_scalar_$r tools/variants/scalar_tail.so --config 5 --steps 20 --warmup 10
done
