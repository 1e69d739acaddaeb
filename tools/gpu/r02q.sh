#!/bin/bash
set -u
O=gpurun_out/r02q; mkdir -p $O
run() { name=$1; pt=$2; tpw=$3; shift 3; BH_PTILE_TPW=$tpw BH_LIB=tools/variants/nolicm_e.so BH_PTILE=$pt timeout -k 10 200 python -u bench.py --no-cpu --steps 48 --warmup 48 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"])')"; }
for r in 1 2; do
run c3D8_tile_$r 0 1
for t in 2 4 8; do run c3D8_static_tpw${t}_$r 2 $t; done
run c3D1_tile_$r 0 1 --frames-per-launch 1
run c3D1_static_tpw2_$r 2 2 --frames-per-launch 1
done
echo done
