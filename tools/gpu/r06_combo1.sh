#!/bin/bash
# round 6: presenter validation + batched frame bench, then rank 0's CU-split unpack probe
set -u -o pipefail
bash tools/gpu/r06_present.sh && bash tools/gpu/r06_rank0.sh
