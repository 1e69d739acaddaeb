#!/bin/bash
# Fixed camera vs an orbiting camera path (every frame its own camera), 8 and 1 frames per launch.
set -u
O=gpurun_out/r02t; mkdir -p $O
run() { name=$1; shift; timeout -k 10 200 python -u bench.py --no-cpu --steps 96 --warmup 96 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"], k["sum_steps"], d["roofline"]["frac"])')"; }
for r in 1 2; do
run fixed_D8_$r
run orbit_D8_$r --camera-path orbit
run fixed_D1_$r --frames-per-launch 1
run orbit_D1_$r --camera-path orbit --frames-per-launch 1
done
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --verify-gather --camera-path orbit --steps 24 --warmup 16 > $O/rehearsal2_orbit.log 2>&1 || exit 14
grep '^{"metric"' $O/rehearsal2_orbit.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rehearsal", d["n_gpus"], d.get("gather_verified_bit_exact"))'
echo done
