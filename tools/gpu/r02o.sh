#!/bin/bash
# Persistent tile schedule (march_ptile_kernel, BH_PTILE=1) with machine LICM off: parity, then A/B
# against the one-wave-per-slot grid, interleaved rounds.
set -u
O=gpurun_out/r02o; mkdir -p $O
BH_LIB=tools/variants/nolicm.so BH_PTILE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_ptile.log 2>&1 || exit 11
run() { name=$1; lib=$2; pt=$3; shift 3; BH_LIB=tools/variants/$lib.so BH_PTILE=$pt timeout -k 10 200 python -u bench.py --no-cpu --steps 96 --warmup 96 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"])')"; }
for r in 1 2; do
 for v in "base 0" "nolicm 0" "nolicm 1"; do
  set -- $v; tag=${1}_pt$2
  run c3D8_${tag}_$r $1 $2
  run c3D1_${tag}_$r $1 $2 --frames-per-launch 1
  run c5D8_${tag}_$r $1 $2 --max-iters 1000 --camera C
  run c5D1_${tag}_$r $1 $2 --max-iters 1000 --camera C --frames-per-launch 1
  run c2D8_${tag}_$r $1 $2 --width 1920 --height 1080 --max-iters 256 --camera B
 done
done
echo done
