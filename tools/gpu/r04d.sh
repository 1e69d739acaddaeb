#!/bin/bash
# round 4: the rsq-seeded reciprocal of the march step -- exhaustive self-test (op 12), the GPU suite,
# interleaved A/B against the v_rcp form (seed0), and the wave-phase probe
set -u
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 150 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_crmath.py > $O/crmath.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || exit 1
for r in 1 2 3; do for v in seed0 seed1; do
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu > $O/h_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu > $O/c2_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 200 python bench.py --config 5 --frames-per-launch 1 --steps 100 --warmup 20 --no-cpu > $O/c5f1_${v}_$r.log 2>&1 || exit 1
done; done
BH_LIB=tools/variants/phases.so timeout -k 10 120 python tools/probe_phases.py > $O/phases.log 2>&1 || exit 1
