#!/bin/bash
# round 5: the root-free step per-term ballots deciding the all-terms test (BH_SDF_TERMS3) -- the march parity suites, then interleaved A/B of
# the driver's bench command against the build without it (variant terms1)
set -u -o pipefail
source tools/gpu/outdir.sh r05 s
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/pytest_march.log 2>&1 || { tail -30 $O/pytest_march.log; exit 1; }
tail -1 $O/pytest_march.log
for rep in 1 2 3; do
  for v in main terms1; do
    L=black_hole_ray_marching_amd/libbh_render.so; if [ $v != main ]; then L=tools/variants/$v.so; fi
    BH_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-extra > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 1
  done
done
python3 - $O <<'PY'
import json, sys, glob
O = sys.argv[1]
for f in sorted(glob.glob(f"{O}/bench_*.json")):
    j = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f.split("/")[-1], j["ms_per_frame"], j["clock"]["mhz"], j["roofline"]["frac"], j["roofline"].get("frac_at_measured_clock"))
PY
