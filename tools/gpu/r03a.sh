#!/bin/bash
# round 3: GPU suite (new graph-contract and clock-probe tests), the driver's bench command and the default bench
set -o pipefail
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_w5.json 2> $O/bench_w5.err || { echo "bench w5 failed"; tail -20 $O/bench_w5.err; exit 1; }
timeout -k 10 240 python bench.py --no-cpu > $O/bench_default.json 2> $O/bench_default.err || { echo "bench default failed"; tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_w5b.json 2> $O/bench_w5b.err || exit 1
python - <<'PY'
import json
for f in ("bench_w5", "bench_default", "bench_w5b"):
    d = json.loads(open(f"gpurun_out/r03a/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_frame"], d["kernel"]["ms_per_frame"], d["roofline"]["frac"], d["roofline"]["frac_at_measured_clock"],
          d["clock"]["mhz"], d.get("single_frame", {}).get("ms_per_frame"), d.get("orbit", {}).get("ms_per_frame"))
PY
