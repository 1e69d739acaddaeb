#!/bin/bash
# Round-2 GPU call F: packed tail step: full GPU suite, chain floor, configs 5 / headline at D=1 and 8.
set -u
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/probe_chain.py --tiles 2 > $O/probe_chain.log 2>&1 || exit 12
for D in 1 8; do
  timeout -k 10 300 python -u bench.py --steps 96 --warmup 96 --no-cpu --frames-per-launch $D > $O/bench_c3_D$D.log 2>&1 || exit 13
  timeout -k 10 300 python -u bench.py --steps 96 --warmup 96 --no-cpu --frames-per-launch $D --max-iters 1000 --camera C > $O/bench_c5_D$D.log 2>&1 || exit 14
done
timeout -k 10 300 python -u tools/probe_shard.py --frames 4096x2048 > $O/probe_shard.log 2>&1 || exit 15
echo done
