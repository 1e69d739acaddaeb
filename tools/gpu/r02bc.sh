#!/bin/bash
# Bloom TapPlan form: bloom parity (incl. 4096x2048) and smoke, then the bloom bench and a kernel trace.
set -u
O=gpurun_out/r02bc; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bloom.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_bloom.log 2>&1 || exit 10
tail -2 $O/pytest_bloom.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 11
tail -1 $O/smoke.log
timeout -k 10 300 python -u tools/bench_bloom.py > $O/bench_bloom.log 2>&1 || exit 12
cat $O/bench_bloom.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_bloom.py --steps 20 > $O/prof.log 2>&1 || exit 13
find $O/prof -name "*kernel_stats.csv" -exec cut -c1-160 {} \;
echo done
