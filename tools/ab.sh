#!/bin/bash
# A/B the exact kernel across library variants in one process each: tools/ab.sh v1 v2 ...
for v in "$@"; do
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --steps 30 --warmup 3 --math ${MATH:-exact} --schedule ${SCHED:-tile} --no-cpu > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel"]["avg_ms"], d["kernel"]["min_ms"], d["value"])')"
done
