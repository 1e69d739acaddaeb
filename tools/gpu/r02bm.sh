#!/bin/bash
# Final confirmation after the bloom Y quad form: full GPU suite, smoke, default +
# driver-style bench, the bloom chain; plus a 2-rank self-launched rehearsal (gather-verified).
set -u
O=gpurun_out/r02bm; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || exit 12
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > $O/bench_w5.log 2>&1 || exit 13
for f in bench_default bench_w5; do tail -1 $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['ms_per_step'], d['value'], d['kernel']['ms_per_frame'], d['roofline']['frac'], d['parity']['bit_exact'], d['parity']['timed_format_bit_exact'], d['clock_settle'])"; done
timeout -k 10 300 python -u tools/bench_bloom.py > $O/bloom.log 2>&1 || exit 14
cat $O/bloom.log
BH_BENCH_REHEARSAL=1 timeout -k 10 300 python -u bench.py --gpus 2 --verify-gather --steps 20 --warmup 5 > $O/rehearsal2.log 2>&1 || exit 15
tail -1 $O/rehearsal2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rehearsal2', d['n_gpus'], d.get('gather_verified_bit_exact'), d['clock_settle'])"
echo done
