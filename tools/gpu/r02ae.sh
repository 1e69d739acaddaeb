#!/bin/bash
# HIP-graph replay and the fast (tolerance) math mode on the current build.
set -u
O=gpurun_out/r02ae; mkdir -p $O
run() { name=$1; shift; timeout -k 10 300 python -u bench.py --steps 96 --warmup 96 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; p=d.get("parity") or {}; print(k["ms_per_frame"], k["avg_ms"], d["value"], p.get("bit_exact"), p.get("fate_nrk_match"), p.get("max_abs_delta_fate_matched"))')"; }
run graph_D8 --graph --no-cpu
run graph_D1 --graph --frames-per-launch 1 --no-cpu
run plain_D1 --frames-per-launch 1 --no-cpu
run fast_D8 --math fast --cpu-reps 1
run fast_D1 --math fast --frames-per-launch 1 --no-cpu
echo done
