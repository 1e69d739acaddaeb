#!/bin/bash
# Round-2 GPU call A: new full-size parity tests, default bench, self-launched 2-rank rehearsal, shard probe.
set -u
O=gpurun_out/r02a; mkdir -p $O
{ cat /sys/fs/cgroup/cpu.max; nproc; python3 -c 'import os; print(len(os.sched_getaffinity(0)))'; } > $O/host.txt 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_configs.log 2>&1 || exit 11
timeout -k 10 300 python -u bench.py --steps 50 --warmup 100 > $O/bench.log 2>&1 || exit 12
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --verify-gather --steps 20 --warmup 10 > $O/rehearsal2.log 2>&1 || exit 13
timeout -k 10 600 python -u tools/probe_shard.py > $O/probe_shard.log 2>&1 || exit 14
echo done
