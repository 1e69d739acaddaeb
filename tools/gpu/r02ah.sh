#!/bin/bash
set -u
O=gpurun_out/r02ah; mkdir -p $O
run() { name=$1; lib=$2; shift 2; BH_LIB=tools/variants/$lib.so timeout -k 10 200 python -u bench.py --no-cpu --steps 96 --warmup 96 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"])')"; }
for r in 1 2 3; do
for v in cur fastnolicm; do
  run fast_D8_${v}_$r $v --math fast
  run fast_D1_${v}_$r $v --math fast --frames-per-launch 1
done
done
echo done
