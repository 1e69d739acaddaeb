#!/bin/bash
set -u
O=gpurun_out/r02v; mkdir -p $O
run() { name=$1; shift; timeout -k 10 200 python -u bench.py --no-cpu --steps 96 --warmup 96 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"], k["sum_steps"])')"; }
run orbit0_D1 --camera-path orbit --orbit-deg 0 --frames-per-launch 1
run orbit02_D1 --camera-path orbit --orbit-deg 0.2 --frames-per-launch 1
run orbit002_D1 --camera-path orbit --orbit-deg 0.02 --frames-per-launch 1
run orbit02_D1_static --camera-path orbit --orbit-deg 0.2 --frames-per-launch 1 --schedule tile-static
run fixed_D1_static --frames-per-launch 1 --schedule tile-static
echo done
