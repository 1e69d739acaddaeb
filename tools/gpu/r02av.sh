#!/bin/bash
# Re-entry confirmation of HEAD (ABI v4, prepared launches): full GPU suite, smoke, the default bench
# and the driver's short-warm-up invocation, then a rocprofv3 kernel trace of the default bench.
set -u
O=gpurun_out/r02av; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 11
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || exit 12
tail -1 $O/bench_default.log
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > $O/bench_w5.log 2>&1 || exit 13
tail -1 $O/bench_w5.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --no-cpu > $O/bench_prof.log 2>&1 || exit 14
echo done
