#!/bin/bash
# round 3: bloom A/B -- the working tree against OLDLIB, interleaved (4096x2048 and 1920x1080), after the GPU suite
set -o pipefail
O=gpurun_out/${OUT:-r03bl}; mkdir -p $O
OLD=${OLDLIB:-tools/variants/prev4.so}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bl() {  # name lib args
  local n=$1 lib=$2; shift 2
  if [ "$lib" = base ]; then timeout -k 10 120 python tools/bench_bloom.py --steps 200 "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  else BH_LIB=$lib timeout -k 10 120 python tools/bench_bloom.py --steps 200 "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; fi
  python -c "import json; [print('$n', x['bloom_schedule'], x['avg_ms']) for x in (json.loads(l) for l in open('$O/$n.json') if l.startswith('{'))]"
}
for r in 1 2 3; do
  bl big_new_$r base
  bl big_old_$r $OLD
  bl hd_new_$r base --width 1920 --height 1080
  bl hd_old_$r $OLD --width 1920 --height 1080
done
