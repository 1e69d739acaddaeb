#!/bin/bash
# BH_MAX_FRAMES 32 (one GPU: 32 frames per launch): GPU suite, smoke, default + short bench, every
# config with its CPU leg, PMC refresh, a 4-rank rehearsal.
set -u
O=gpurun_out/r02ap; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 11
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || exit 13
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --no-cpu > $O/bench_w5.log 2>&1 || exit 14
timeout -k 10 900 bash tools/configs.sh > $O/configs.log 2>&1 || exit 15
timeout -k 10 900 bash tools/gpu/pmc_configs.sh r02i > $O/pmc.log 2>&1 || exit 16
BH_BENCH_REHEARSAL=1 timeout -k 10 400 python -u bench.py --gpus 4 --verify-gather --steps 16 --warmup 8 > $O/rehearsal4.log 2>&1 || exit 17
echo done
