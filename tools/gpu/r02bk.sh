#!/bin/bash
# A/B: iterations before a wave raises its priority and starts the cycle watch (PRIO_ITERS 36/48/60/96).
set -u
O=gpurun_out/r02bk; mkdir -p $O
timeout -k 10 500 bash tools/ab_interleaved.sh 2 "--steps 64 --warmup 64" p48 p36 p60 p96 > $O/c3.log 2>&1 || exit 1
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--config 2 --steps 128 --warmup 64" p48 p36 p60 p96 > $O/c2.log 2>&1 || exit 2
timeout -k 10 300 bash tools/ab_interleaved.sh 2 "--config 5 --steps 64 --warmup 64" p48 p36 p60 p96 > $O/c5.log 2>&1 || exit 3
for f in c3 c2 c5; do echo "== $f"; cat $O/$f.log; done
