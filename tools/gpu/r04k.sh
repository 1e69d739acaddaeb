#!/bin/bash
# round 4: the yq tile's row-pair shift (bank conflicts) -- bloom GPU tests, interleaved A/B against the old
# layout at 4096x2048, and the bloom PMC of the new one
set -u
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom.log 2>&1 || exit 1
for r in 1 2 3; do for v in yq_old yq_new; do
  BH_LIB=tools/variants/$v.so timeout -k 10 120 python tools/bench_bloom.py --steps 50 > $O/ab_${v}_$r.log 2>&1 || exit 1
done; done
OUT=r04k/bloom_pmc_4096 bash tools/gpu/bloom_pmc.sh 4096 2048 > $O/bloom_pmc.log 2>&1 || exit 1
# per-tile render cost against the shard count (the N>1 model's render term): n = 1 in the packed layout
timeout -k 10 300 python tools/probe_rank0.py --n 1,2,8 --D 16 --rows 64 --root-ratio 1 --transport rgbm14 --it 8 > $O/rank0_n1.jsonl 2> $O/rank0_n1.err || exit 1
timeout -k 10 200 python bench.py --frames-per-launch 16 --steps 20 --warmup 5 --no-cpu --no-extra > $O/h_D16.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-extra > $O/h_D32.log 2>&1 || exit 1
