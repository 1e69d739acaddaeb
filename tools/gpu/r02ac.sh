#!/bin/bash
# Costs recorded by a launch's first vs last frame: fixed camera and orbit path, 8 frames per launch.
set -u
O=gpurun_out/r02ac; mkdir -p $O
BH_LIB=tools/variants/lastf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -k "render_frames or partition" --timeout 200 --timeout-method thread > $O/pytest_lastf.log 2>&1 || exit 11
run() { name=$1; lib=$2; shift 2; BH_LIB=tools/variants/$lib.so timeout -k 10 200 python -u bench.py --no-cpu --steps 96 --warmup 96 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"])')"; }
for r in 1 2; do
for v in firstf lastf; do
  run fixed_D8_${v}_$r $v
  run orbit_D8_${v}_$r $v --camera-path orbit
  run orbit2_D8_${v}_$r $v --camera-path orbit --orbit-deg 0.05
done
done
echo done
