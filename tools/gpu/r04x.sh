#!/bin/bash
# round 4: the GPU suite on the final tree (new parity cases at the root-free step's gates), smoke, then
# the bloom A/B of r04fix
set -u
O=gpurun_out/r04x; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
bash tools/gpu/r04fix.sh || exit 1
