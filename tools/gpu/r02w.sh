#!/bin/bash
# Dilated order costs (order_cost_kernel): parity, then fixed vs orbit camera, dilation on / off.
set -u
O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 11
run() { name=$1; dl=$2; shift 2; BH_ORDER_DILATE=$dl timeout -k 10 200 python -u bench.py --no-cpu --steps 96 --warmup 96 "$@" > $O/$name.log 2>&1 || exit 12; echo "$name $(grep '^{"metric"' $O/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"])')"; }
for r in 1 2; do
for dl in 0 1; do
run fixed_D8_dl${dl}_$r $dl
run fixed_D1_dl${dl}_$r $dl --frames-per-launch 1
run orbit_D8_dl${dl}_$r $dl --camera-path orbit
run orbit_D1_dl${dl}_$r $dl --camera-path orbit --frames-per-launch 1
run c5_D1_dl${dl}_$r $dl --max-iters 1000 --camera C --frames-per-launch 1
done
done
for dl in 0 1; do BH_ORDER_DILATE=$dl timeout -k 10 300 python -u tools/probe_shard.py --frames 4096x2048 --shards 8 > $O/shard_dl$dl.log 2>&1 || exit 13; done
echo done
