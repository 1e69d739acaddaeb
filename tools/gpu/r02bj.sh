#!/bin/bash
# A/B: decode table loaded by LDS DMA at wave start and awaited only before the shading (lutlate) vs
# the load + barrier at wave start (base); interleaved; parity of the variant on the GPU suite's
# parity tests first.
set -u
O=gpurun_out/r02bj; mkdir -p $O
BH_LIB=tools/variants/lutlate.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_lutlate.log 2>&1 || exit 1
tail -1 $O/pytest_lutlate.log
timeout -k 10 500 bash tools/ab_interleaved.sh 3 "--steps 64 --warmup 64" base lutlate > $O/c3.log 2>&1 || exit 2
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--config 2 --steps 128 --warmup 64" base lutlate > $O/c2.log 2>&1 || exit 3
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--config 5 --steps 64 --warmup 64" base lutlate > $O/c5.log 2>&1 || exit 4
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--config 1 --steps 1024 --warmup 512" base lutlate > $O/c1.log 2>&1 || exit 5
for f in c3 c2 c5 c1; do echo "== $f"; cat $O/$f.log; done
