#!/bin/bash
set -u
O=gpurun_out/r02p; mkdir -p $O
run() { name=$1; lib=$2; pt=$3; pc=$4; shift 4; BH_PTILE_PER_CU=$pc BH_LIB=tools/variants/$lib.so BH_PTILE=$pt timeout -k 10 200 python -u bench.py --no-cpu --steps 48 --warmup 48 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"])')"; }
for pc in 2 4 8 9; do run c3D8_pt_pc$pc nolicm_e 1 $pc; done
run c3D8_tile nolicm_e 0 8
run c5D1_tile nolicm_e 0 8 --max-iters 1000 --camera C --frames-per-launch 1
echo done
