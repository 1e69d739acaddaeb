#!/bin/bash
# round 6: parity of the march (configs, parity) then the camera tail probe and the headline bench
set -u -o pipefail
source tools/gpu/outdir.sh r06 tail
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_present.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cap in 512 1000; do
  timeout -k 10 200 python -u tools/probe_camera_tail.py --cameras A,B,C --max-iters $cap --reps 8 >> $O/camtail.log 2>&1 || { tail -30 $O/camtail.log; exit 1; }
done
grep camera $O/camtail.log
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
