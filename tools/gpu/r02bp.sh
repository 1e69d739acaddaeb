#!/bin/bash
# A/B: decode tables and cycle history sharing one 4 KiB LDS block per one-wave workgroup (union; tail
# waves reload the tables) vs separate 1 + 4 KiB (base); parity of the variant first.
set -u
O=gpurun_out/r02bp; mkdir -p $O
BH_LIB=tools/variants/union.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_random.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_union.log 2>&1 || exit 1
tail -1 $O/pytest_union.log
timeout -k 10 500 bash tools/ab_interleaved.sh 3 "--steps 64 --warmup 64" base union > $O/c3.log 2>&1 || exit 2
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--config 2 --steps 128 --warmup 64" base union > $O/c2.log 2>&1 || exit 3
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--config 5 --steps 64 --warmup 64" base union > $O/c5.log 2>&1 || exit 4
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--frames-per-launch 1 --steps 64 --warmup 64" base union > $O/c3_D1.log 2>&1 || exit 5
for f in c3 c2 c5 c3_D1; do echo "== $f"; cat $O/$f.log; done
