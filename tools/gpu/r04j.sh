#!/bin/bash
# round 4: GPU suite on the kept root-free form; rank-0 probes with the unpack stream at normal / high
# priority; a 2- and 3-rank rehearsal through the bench (calibration grid, priority stream), gather-verified
set -u
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 400 python tools/probe_rank0.py --n 8,4,2 --D 16 --rows 64 --root-ratio auto,1 --side-priority 0,-1 --transport rgbm14 --it 8 > $O/rank0.jsonl 2> $O/rank0.err || exit 1
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --verify-gather --steps 4 --warmup 2 --no-cpu > $O/reh2.json 2> $O/reh2.err || exit 1
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 3 --verify-gather --steps 4 --warmup 2 --no-cpu > $O/reh3.json 2> $O/reh3.err || exit 1
