#!/bin/bash
# round 5: validation of the current build -- the whole GPU suite, smoke, the driver's bench command, the
# bloom sizes, 2- and 3-rank rehearsals
set -u -o pipefail
source tools/gpu/outdir.sh r05 ${TAG:-n}
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
for s in "1920 1080" "1280 720" "4096 2048"; do
  set -- $s
  timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --steps 200 >> $O/bloom.log 2>>$O/bloom.err || exit 1
done
BH_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --verify-gather --steps 4 --warmup 2 --no-cpu > $O/reh2.json 2> $O/reh2.err || exit 1
BH_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 3 --verify-gather --steps 4 --warmup 2 --no-cpu > $O/reh3.json 2> $O/reh3.err || exit 1
python3 - $O <<'PY'
import json, sys
O = sys.argv[1]
j = json.loads([l for l in open(f"{O}/bench.json") if l.startswith("{")][-1])
print("bench", j["ms_per_frame"], j["value"], j["clock"]["mhz"], j["roofline"]["frac"], j["roofline"].get("frac_at_measured_clock"),
      j.get("parity", {}).get("max_abs_delta"), "single", j["single_frame"]["ms_per_frame"], "orbit", j["orbit"]["ms_per_frame"],
      "cpu", j["cpu_baseline"]["value"])
for l in open(f"{O}/bloom.log"):
    if l.startswith("{"):
        b = json.loads(l); print("bloom", b["bloom_schedule"], b["width"], b["avg_ms"])
for f in ("reh2.json", "reh3.json"):
    r = json.loads([l for l in open(f"{O}/{f}") if l.startswith("{")][-1]); print(f, r["n_gpus"], r.get("gather_verified_bit_exact"))
PY
