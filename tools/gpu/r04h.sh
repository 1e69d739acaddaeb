#!/bin/bash
# round 4: GPU suite on the final root-free step (fcmp lane mask), A/B skip0 vs skip1 (headline, config 1),
# config 1 fixed cost PMC (cap 64 / 1 / 2), bloom PMC at 1920x1080 and 4096x2048, rank-0 probes for N>1
set -u
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || exit 1
BH_LIB=tools/variants/diag.so timeout -k 10 120 python tools/diag_slow.py > $O/diag.log 2>&1 || exit 1
cp black_hole_ray_marching_amd/libbh_render.so tools/variants/skip1.so
for r in 1 2; do for v in skip0 skip1; do
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu > $O/h_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --config 1 --steps 20 --warmup 5 --no-cpu > $O/c1_${v}_$r.log 2>&1 || exit 1
done; done
bash tools/gpu/pmc_configs.sh r04h c1 c1cap1 c1cap2 > $O/pmc.log 2>&1 || exit 1
OUT=r04h/bloom_pmc_1920 bash tools/gpu/bloom_pmc.sh 1920 1080 > $O/bloom_pmc.log 2>&1 || exit 1
OUT=r04h/bloom_pmc_4096 bash tools/gpu/bloom_pmc.sh 4096 2048 >> $O/bloom_pmc.log 2>&1 || exit 1
for D in 16 32; do
  timeout -k 10 300 python tools/probe_rank0.py --n 2,4,8 --D $D --rows 64 --root-ratio auto,1 --transport rgbm14 --it 8 >> $O/rank0.jsonl 2> $O/rank0_$D.err || exit 1
done
