#!/bin/bash
# Every single-GPU BASELINE.json config through bench.py (exact math, with the CPU leg = parity +
# cpu_baseline): -> gpurun_out/configs/*.json.  Config 4 (8 GPUs) is the driver's.
mkdir -p gpurun_out/configs
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/configs/$n.log 2>&1 || exit 1; grep '^{"metric"' gpurun_out/configs/$n.log > gpurun_out/configs/$n.json; }
run c1_256x256_cap64_nosurf --width 256 --height 256 --max-iters 64 --surfaces off
run c2_1920x1080_cap256_B --width 1920 --height 1080 --max-iters 256 --camera B
run c3_4096x2048_cap512_A
run c3_4096x2048_cap512_B --camera B
run c5_4096x2048_cap1000_C --max-iters 1000 --camera C
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/configs/*.json")):
    d = json.load(open(f)); k = d["kernel"]; par = d.get("parity") or {}
    print(f"{os.path.basename(f)[:-5]:28s} {d['value']:9.1f} Mpix/s  kernel {k['avg_ms']:.4f} ms  fps {k['frames_per_s']:8.1f}  "
          f"bit_exact {par.get('bit_exact')}  cpu {d['cpu_baseline']['value'] if d.get('cpu_baseline') else None} Mpix/s")
PY
