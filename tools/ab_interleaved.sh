#!/bin/bash
# A/B library variants on one box, interleaved over rounds (clock drift hits every variant alike):
#   tools/ab_interleaved.sh ROUNDS "bench args" v1 v2 ...   -> gpurun_out/ab/<variant>_<round>.json
set -u
R=$1; ARGS=$2; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for v in "$@"; do
    BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --no-cpu $ARGS > gpurun_out/ab/${v}_$r.log 2>&1 || exit 1
    grep '^{"metric"' gpurun_out/ab/${v}_$r.log > gpurun_out/ab/${v}_$r.json
    echo "$r $v $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); k=d["kernel"]; print(k["ms_per_frame"], k["avg_ms"], d["value"])' gpurun_out/ab/${v}_$r.json)"
  done
done
