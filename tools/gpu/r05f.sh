#!/bin/bash
# round 5: the whole GPU suite, smoke and the driver's bench command on the current build (in-block fix),
# the bloom sizes, then the one-frame-per-launch experiments: the latency build at one frame, a kernel trace
# of one-frame launches (order kernel, march kernel and the gaps between them)
set -u
source tools/gpu/outdir.sh r05 f
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
for s in "1920 1080" "1280 720" "4096 2048"; do
  set -- $s
  timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --steps 100 --schedule auto >> $O/bloom.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 5 --variant latency > $O/bench_latency.json 2> $O/bench_latency.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 5 --variant issue > $O/bench_issue.json 2> $O/bench_issue.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_d1 -o run -- python bench.py --no-cpu --no-extra --steps 30 --warmup 10 --frames-per-launch 1 > $O/bench_d1.json 2> $O/bench_d1.err || exit 1
python3 - $O <<'PY'
import json, sys
O = sys.argv[1]
for f in ("bench.json", "bench_latency.json", "bench_issue.json", "bench_d1.json"):
    try:
        j = json.loads([l for l in open(f"{O}/{f}") if l.startswith("{")][-1])
    except Exception as e:
        print(f, "no line", e); continue
    print(f, j["ms_per_frame"], j.get("clock", {}).get("mhz"), j["roofline"]["frac"], j.get("parity", {}).get("bit_exact"),
          "single", (j.get("single_frame") or {}).get("ms_per_frame"), (j.get("single_frame") or {}).get("kernel_ms_per_frame"),
          "orbit", (j.get("orbit") or {}).get("ms_per_frame"))
PY
