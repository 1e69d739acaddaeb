#!/bin/bash
# A/B the march kernel across library variants, one process each: tools/ab.sh v1 v2 ...
#   env: MATH (exact|fast), SCHED (tile|...), STEPS (30), EXTRA (more bench.py args)
for v in "$@"; do
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --steps ${STEPS:-30} --warmup 3 --math ${MATH:-exact} \
    --schedule ${SCHED:-tile} --no-cpu $EXTRA > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo "$v $EXTRA $(tail -1 gpurun_out/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel"]["avg_ms"], d["kernel"]["min_ms"], d["value"])')"
done
