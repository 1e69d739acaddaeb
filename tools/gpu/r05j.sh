#!/bin/bash
# round 5: bloom parity with the final epilogue's fix opt-in (its switches in child processes), the chain at
# the three sizes
set -u -o pipefail
source tools/gpu/outdir.sh r05 j
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || { tail -30 $O/pytest_bloom.log; exit 1; }
tail -1 $O/pytest_bloom.log
for s in "1920 1080" "1280 720" "4096 2048"; do
  set -- $s
  timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --steps 200 --schedule auto >> $O/bloom.log 2>>$O/bloom.err || exit 1
done
python3 -c "
import json,sys
for l in open('$O/bloom.log'):
    j=json.loads(l); print(j['width'], j['height'], j['avg_ms'], j['min_ms'])"
