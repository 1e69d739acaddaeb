#!/bin/bash
# round 3: bloom literal passes' short forms (texel-centre copies/remixes, 2:1 half-weight downsamples):
# bloom GPU tests, then the chain at 4096x2048 (fused + literal) and 1920x1080 (not exact: literal), vs HEAD
set -o pipefail
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bloom.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
b() {  # name lib args
  local n=$1 lib=$2; shift 2
  if [ "$lib" = base ]; then timeout -k 10 120 python tools/bench_bloom.py --steps 100 "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  else BH_LIB=$lib timeout -k 10 120 python tools/bench_bloom.py --steps 100 "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; fi
  python -c "import json; d=[json.loads(l) for l in open('$O/$n.json') if l.startswith('{')]; print('$n', *[(x['bloom_schedule'], x['avg_ms']) for x in d])"
}
for r in 1 2; do
  b big_new_$r base
  b big_old_$r tools/variants/head.so
  b hd_new_$r base --width 1920 --height 1080
  b hd_old_$r tools/variants/head.so --width 1920 --height 1080
done
