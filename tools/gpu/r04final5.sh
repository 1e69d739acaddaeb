#!/bin/bash
# round 4, final build (bloom fix-up gather, paired downsamples, 8-byte plan entries): GPU suite, smoke, the driver's bench
# command, its rocprofv3 kernel-trace summary, bloom at the three frame sizes
set -u
O=gpurun_out/r04final5; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_prof -o run -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-extra > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
for s in "1920 1080" "1280 720" "4096 2048"; do
  set -- $s
  timeout -k 10 120 python tools/bench_bloom.py --width $1 --height $2 --steps 50 >> $O/bloom.log 2>&1 || exit 1
done
