#!/bin/bash
set -u
O=gpurun_out/r02ag; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_random.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_random.log 2>&1 || exit 11
echo done
