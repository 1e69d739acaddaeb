#!/bin/bash
# Frames per launch on the one-wave-workgroup build: 32 / 64 / 128, interleaved, headline + cap 1000.
set -u
O=gpurun_out/r02bl; mkdir -p $O
for r in 1 2; do
  for D in 32 64 128; do
    timeout -k 10 200 python bench.py --no-cpu --steps 128 --warmup 128 --frames-per-launch $D > $O/c3_D${D}_$r.log 2>&1 || exit 1
    echo "c3 $r $D $(tail -1 $O/c3_D${D}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel"]["ms_per_frame"], d["ms_per_step"])')"
    timeout -k 10 200 python bench.py --no-cpu --config 5 --steps 128 --warmup 128 --frames-per-launch $D > $O/c5_D${D}_$r.log 2>&1 || exit 2
    echo "c5 $r $D $(tail -1 $O/c5_D${D}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel"]["ms_per_frame"], d["ms_per_step"])')"
  done
done
