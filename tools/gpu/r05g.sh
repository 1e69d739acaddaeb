#!/bin/bash
# round 5: repeated frames skip the order build (bh_host.cpp OrderState keys) -- the order / graph tests, then
# the driver's bench command with and without the skip (BH_ORDER_ALWAYS=1), interleaved
set -u
source tools/gpu/outdir.sh r05 g
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "order or graph or repeated or stream or partition" > $O/pytest_order.log 2>&1 || { tail -30 $O/pytest_order.log; exit 1; }
tail -1 $O/pytest_order.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_skip_$rep.json 2> $O/bench_skip_$rep.err || exit 1
  BH_ORDER_ALWAYS=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_always_$rep.json 2> $O/bench_always_$rep.err || exit 1
done
python3 - $O <<'PY'
import json, sys, glob
O = sys.argv[1]
for f in sorted(glob.glob(f"{O}/bench_*.json")):
    j = json.loads([l for l in open(f) if l.startswith("{")][-1])
    sf, ob = j.get("single_frame") or {}, j.get("orbit") or {}
    print(f.split("/")[-1], j["ms_per_frame"], j["clock"]["mhz"], "single", sf.get("ms_per_frame"), sf.get("kernel_ms_per_frame"),
          sf.get("clock_mhz"), "orbit", ob.get("ms_per_frame"))
PY
