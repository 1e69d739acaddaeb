#!/bin/bash
# Round-2 GPU call C: multi-frame launches: GPU tests, bench at D = 1/2/4/8, rehearsal, in-flight probe.
set -u
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_configs.log 2>&1 || exit 11
for D in 1 2 4 8; do
  timeout -k 10 300 python -u bench.py --steps 96 --warmup 96 --no-cpu --frames-per-launch $D > $O/bench_D$D.log 2>&1 || exit 12
done
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --verify-gather --steps 24 --warmup 8 --frames-per-launch 4 > $O/rehearsal2_D4.log 2>&1 || exit 13
timeout -k 10 600 python -u tools/probe_inflight.py --modes batch --depths 1,2,4,8 > $O/probe_inflight.log 2>&1 || exit 14
echo done
