#!/bin/bash
# RCCL dry run: the N>1 code path at one rank over a real nccl process group (test + full-size bench).
set -u
O=gpurun_out/r02al; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bench_launch.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest_dry.log 2>&1 || exit 11
NCCL_DEBUG=WARN timeout -k 10 300 python -u bench.py --rccl-dry-run --verify-gather --steps 48 --warmup 96 > $O/bench_dry_full.log 2>&1 || exit 12
echo done
