#!/bin/bash
# Which exact build for configs 1 and 2 at 32 frames per launch: source-order (issue) vs scheduled (latency).
set -u
O=gpurun_out/r02at; mkdir -p $O
for C in 1 2; do
  for rep in 1 2 3; do
    for V in issue latency; do
      timeout -k 10 200 python -u bench.py --config $C --no-cpu --steps 160 --warmup 320 --variant $V > $O/c${C}_${V}_r$rep.log 2>&1 || exit 1
      tail -1 $O/c${C}_${V}_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c$C $V r$rep', d['ms_per_step'], d['kernel']['ms_per_frame'], d['kernel']['name'])"
    done
  done
done
echo done
