#!/bin/bash
# Variant (issue-order vs latency build) per workload at 8 / 1 frames per launch.
set -u
O=gpurun_out/r02h; mkdir -p $O
run() { n=$1; shift; timeout -k 10 200 python -u bench.py --no-cpu --steps 96 --warmup 96 "$@" > $O/$n.log 2>&1 || exit 11; echo "$n $(grep '^{"metric"' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"])')"; }
for r in 1 2; do
for v in issue latency; do
  run c3_D8_$v$r --variant $v
  run c5_D8_$v$r --max-iters 1000 --camera C --variant $v
  run c2_D8_$v$r --width 1920 --height 1080 --max-iters 256 --camera B --variant $v
  run c1_D8_$v$r --width 256 --height 256 --max-iters 64 --surfaces off --variant $v
  run c5_D1_$v$r --max-iters 1000 --camera C --variant $v --frames-per-launch 1
  run c2_D1_$v$r --width 1920 --height 1080 --max-iters 256 --camera B --variant $v --frames-per-launch 1
done
done
for v in issue latency; do
  timeout -k 10 300 python -u tools/probe_inflight.py --modes batch --shards 4,8 --depths 1,8 --variant $v > $O/inflight_$v.log 2>&1 || exit 12
done
echo done
