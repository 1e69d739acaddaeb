#!/bin/bash
# round 5: rocprofv3 kernel trace + PMC passes of the current build's bench (headline, one frame per launch,
# config 2), and the driver's bench command with the single-frame leg's bare wall pass
set -u -o pipefail
source tools/gpu/outdir.sh r05 p
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
bash tools/gpu/pmc_configs.sh r05p c3A c3A_D1 c2 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
tail -3 $O/pmc.log
python3 - $O <<'PY'
import json, sys
O = sys.argv[1]
j = json.loads([l for l in open(f"{O}/bench.json") if l.startswith("{")][-1])
print("bench", j["ms_per_frame"], j["value"], j["clock"]["mhz"], j["roofline"]["frac"], j["roofline"].get("frac_at_measured_clock"))
print("single", j["single_frame"]); print("orbit", j["orbit"])
PY
