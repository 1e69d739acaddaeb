#!/bin/bash
# round 4: 8-byte plan entries in the quad up pass's LDS (BH_BLOOM_SEPQ_E8: 73-85 VGPRs instead of 89-93,
# 4 KiB less LDS) -- bloom GPU tests with the variant, interleaved A/B against the same build without
set -u
O=gpurun_out/r04e8; mkdir -p $O
BH_LIB=tools/variants/e8.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_bloom.py > $O/pytest_bloom_e8.log 2>&1 || exit 1
for r in 1 2 3; do for v in bbase e8; do
  BH_LIB=tools/variants/$v.so timeout -k 10 120 python tools/bench_bloom.py --width 1920 --height 1080 --steps 50 --schedule auto > $O/ab1920_${v}_$r.log 2>&1 || exit 1
  BH_LIB=tools/variants/$v.so timeout -k 10 120 python tools/bench_bloom.py --width 1280 --height 720 --steps 50 --schedule auto > $O/ab1280_${v}_$r.log 2>&1 || exit 1
done; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
BH_LIB=tools/variants/e8.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace1920 -o run -- python tools/bench_bloom.py --width 1920 --height 1080 --steps 20 --schedule auto > $O/trace1920.log 2>&1 || exit 1
