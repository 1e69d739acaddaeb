#!/bin/bash
# Loop-kept n_rk (exit code per lane): parity suites, A/B uni vs ex.
set -u
O=gpurun_out/r02bb; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 10
tail -2 $O/pytest.log
timeout -k 10 800 bash tools/ab_interleaved.sh 4 "--steps 128 --warmup 256" uni ex > $O/ab_headline.log 2>&1 || exit 11
cat $O/ab_headline.log
timeout -k 10 600 bash tools/ab_interleaved.sh 3 "--config 2 --steps 256 --warmup 256" uni ex > $O/ab_c2.log 2>&1 || exit 12
cat $O/ab_c2.log
timeout -k 10 600 bash tools/ab_interleaved.sh 3 "--config 5 --steps 128 --warmup 256" uni ex > $O/ab_c5.log 2>&1 || exit 13
cat $O/ab_c5.log
echo done
