#!/bin/bash
# Hazard-slot filling (no s_nop after v_rsq / v_rcp in the step): parity, then interleaved A/B.
set -u
O=gpurun_out/r02z; mkdir -p $O
BH_LIB=tools/variants/nonop.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_nonop.log 2>&1 || exit 11
run() { name=$1; lib=$2; shift 2; BH_LIB=tools/variants/$lib.so timeout -k 10 200 python -u bench.py --no-cpu --steps 96 --warmup 96 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"])')"; }
for r in 1 2 3; do
for v in basenop nonop; do
  run c3D8_${v}_$r $v
  run c3D1_${v}_$r $v --frames-per-launch 1
  run c5D1_${v}_$r $v --max-iters 1000 --camera C --frames-per-launch 1
  run c2D8_${v}_$r $v --width 1920 --height 1080 --max-iters 256 --camera B
done
done
echo done
