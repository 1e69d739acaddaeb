#!/bin/bash
# round 3 final validation: the GPU suite, smoke(), the default bench, the driver's command, a 2-rank
# rehearsal with gather verification, and the bloom chain -- each under its own time limit
set -o pipefail
O=gpurun_out/${OUT:-r03final}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -10 $O/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || { echo "driver cmd failed"; tail -10 $O/bench_driver_cmd.err; exit 1; }
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --verify-gather --no-cpu > $O/rehearsal2.json 2> $O/rehearsal2.err || { echo "rehearsal failed"; tail -10 $O/rehearsal2.err; exit 1; }
timeout -k 10 120 python tools/bench_bloom.py --steps 200 > $O/bloom.json 2> $O/bloom.err || { echo "bloom failed"; tail -10 $O/bloom.err; exit 1; }
python - <<'PY'
import json
import os; O = "gpurun_out/" + os.environ.get("OUT", "r03final")
for n in ("bench_default", "bench_driver_cmd", "rehearsal2"):
    d = json.loads(open(f"{O}/{n}.json").read().strip().splitlines()[-1])
    c = d.get("clock") or {}
    print(n, d["value"], d["unit"], "ms/frame", d.get("ms_per_frame"), "clock", c.get("mhz"), c.get("per_xcd_mhz"),
          "frac", d.get("roofline", {}).get("frac"), "parity", (d.get("parity") or {}).get("bit_exact"),
          "gather_ok", d.get("gather_verified_bit_exact"), "single", (d.get("single_frame") or {}).get("ms_per_frame"),
          "orbit", (d.get("orbit") or {}).get("ms_per_frame"))
for l in open(f"{O}/bloom.json"):
    if l.startswith("{"):
        x = json.loads(l); print("bloom", x["bloom_schedule"], x["avg_ms"])
PY
