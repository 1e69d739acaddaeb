#!/bin/bash
# Validation of the current build on one GPU (run through gpurun from the repo root):
#   bash tools/gpu/validate.sh ROUND [quick]
# the full GPU test suite, smoke(), the driver's bench command, the bench under the rocprofv3 kernel trace
# (its stats next to the bench line), the bloom chain at the three display sizes, the app frame (serial vs
# pipelined, tools/bench_frame.py) and the 2- and 3-rank rehearsals (all ranks on cuda:0 over gloo,
# gather-verified).  `quick`: no test suite.  Output: gpurun_out/ROUND/validate/<time>/
set -u -o pipefail
source tools/gpu/outdir.sh "${1:?round}" validate
MODE=${2:-full}
if [ "$MODE" != quick ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("bench", d["ms_per_frame"], d["value"], d["clock"]["mhz"], d["roofline"]["frac"], d["roofline"]["frac_at_measured_clock"],
      "single", d["single_frame"]["ms_per_frame"], "orbit", d["orbit"]["ms_per_frame"],
      "single_orbit", (d.get("single_frame_orbit") or {}).get("ms_per_frame"), "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
mkdir -p $O/trace
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-extra > $GRAFT_REPO_ROOT/$O/trace.log 2>&1) || { tail -20 $O/trace.log; exit 1; }
grep -h '^{"metric"' $O/trace.log > $O/trace_bench_line.json || true
for s in "1920 1080" "1280 720" "4096 2048"; do
  set -- $s
  timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --schedule auto --steps 200 >> $O/bloom.log 2>> $O/bloom.err || { tail -20 $O/bloom.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/bloom.log'):
    d = json.loads(l); print('bloom', d['width'], d['height'], d['avg_ms'])"
timeout -k 10 400 python -u tools/bench_frame.py --variants "" --cus "" > $O/frame.log 2>&1 || { tail -30 $O/frame.log; exit 1; }
grep width $O/frame.log | cut -c1-400
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --steps 4 --warmup 2 --verify-gather > $O/reh2.json 2> $O/reh2.err || { tail -20 $O/reh2.err; exit 1; }
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 3 --steps 4 --warmup 2 --verify-gather --fmt bgra8 > $O/reh3.json 2> $O/reh3.err || { tail -20 $O/reh3.err; exit 1; }
python3 - $O <<'PY'
import json, sys
for f in ("reh2", "reh3"):
    d = json.loads(open(f"{sys.argv[1]}/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d.get("gather_verified_bit_exact"), d["config"]["workload"][:160])
PY
echo "validate ok: $O"
