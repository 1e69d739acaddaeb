#!/bin/bash
# Per-frame cost of everything but the RK loop: the headline frame at caps 1 / 2 / 4 / 8 / 16 (8 frames
# per launch), and the fast mode's parity at full size.
set -u
O=gpurun_out/r02af; mkdir -p $O
run() { name=$1; shift; timeout -k 10 300 python -u bench.py --steps 96 --warmup 96 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; p=d.get("parity") or {}; print(k["ms_per_frame"], k["avg_ms"], d["value"], k["sum_steps"], p.get("bit_exact"), p.get("fate_nrk_match"), p.get("max_abs_delta_fate_matched_uncapped"))')"; }
for c in 1 2 4 8 16 512; do run cap$c --max-iters $c --no-cpu; done
run fast_D8 --math fast --cpu-reps 1
echo done
