#!/bin/bash
# Tile cost for the order = max executed steps (firstf, as built) vs max loop iterations n_rk (nrkcost).
set -u
O=gpurun_out/r02ad; mkdir -p $O
run() { name=$1; lib=$2; shift 2; BH_LIB=tools/variants/$lib.so timeout -k 10 200 python -u bench.py --no-cpu --steps 96 --warmup 96 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"])')"; }
for r in 1 2; do
for v in firstf nrkcost; do
  run fixed_D8_${v}_$r $v
  run fixed_D1_${v}_$r $v --frames-per-launch 1
  run orbit_D8_${v}_$r $v --camera-path orbit
  run orbit_D1_${v}_$r $v --camera-path orbit --frames-per-launch 1
  run c5_D1_${v}_$r $v --max-iters 1000 --camera C --frames-per-launch 1
done
done
echo done
