#!/bin/bash
# Bench every schedule x math mode (1 GPU, headline config) -> gpurun_out/sweep/*.json + a table.
#   tools/sweep.sh [steps]
S=${1:-100}
mkdir -p gpurun_out/sweep
for m in exact fast; do
  for s in tile tile-static pair persistent; do
    timeout -k 10 200 python bench.py --steps $S --warmup 5 --math $m --schedule $s --no-cpu \
      > gpurun_out/sweep/${m}_${s}.log 2>&1 || exit 1
    tail -1 gpurun_out/sweep/${m}_${s}.log > gpurun_out/sweep/${m}_${s}.json
  done
done
for c in 64 1000; do
  timeout -k 10 200 python bench.py --steps $S --warmup 5 --math exact --max-iters $c --no-cpu \
    > gpurun_out/sweep/exact_tile_cap$c.log 2>&1 || exit 1
  tail -1 gpurun_out/sweep/exact_tile_cap$c.log > gpurun_out/sweep/exact_tile_cap$c.json
done
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/sweep/*.json")):
    d = json.load(open(f)); k = d["kernel"]
    print(f"{os.path.basename(f)[:-5]:24s} avg {k['avg_ms']:.4f} ms  min {k['min_ms']:.4f}  {d['value']:9.1f} Mpix/s  fps {k['frames_per_s']:7.1f}  frac {d['roofline']['frac']:.4f}")
PY
