#!/bin/bash
# The driver's invocation (--warmup 5 --steps 20) with settle 100 / 300 / 1000 ms, interleaved, vs the
# default run's steady state (300 warm-up, 100 timed).
set -u
O=gpurun_out/r02bn; mkdir -p $O
for r in 1 2 3; do
  for S in 100 300 1000; do
    timeout -k 10 200 python bench.py --no-cpu --warmup 5 --steps 20 --settle-ms $S > $O/w5_s${S}_$r.log 2>&1 || exit 1
    echo "w5 settle $S r$r $(tail -1 $O/w5_s${S}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel"]["ms_per_frame"])')"
  done
  timeout -k 10 200 python bench.py --no-cpu > $O/default_$r.log 2>&1 || exit 2
  echo "default r$r $(tail -1 $O/default_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel"]["ms_per_frame"])')"
done
