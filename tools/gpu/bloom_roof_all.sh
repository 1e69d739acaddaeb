#!/bin/bash
# The bloom chain's per-kernel PMC roofline at the display sizes (tools/gpu/bloom_roofline.sh per size, then
# tools/bloom_roofline.py with the chain time of a bench_bloom run):  bash tools/gpu/bloom_roof_all.sh
#   -> gpurun_out/r06/bloom_roof/<W>/roofline.json (copied to profiles/r06/bloom_roof/roofline<W>.json)
set -u -o pipefail
for s in "1920 1080" "1280 720" "4096 2048" "3840 2160"; do
  set -- $s
  D=gpurun_out/r06/bloom_roof/$1
  bash tools/gpu/bloom_roofline.sh $1 $2 $D || exit 1
  timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --schedule auto --steps 200 > $D/bench.log 2>/dev/null || exit 1
  MS=$(python3 -c "import json,sys; print(json.loads(open('$D/bench.log').read().strip().splitlines()[-1])['avg_ms'])")
  python3 tools/bloom_roofline.py --width $1 --height $2 --pmc $D --chain-ms $MS > $D/roofline.json || exit 1
  echo "$1x$2 $MS"
done
