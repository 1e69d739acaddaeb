#!/bin/bash
# round 6: rank 0's render + unpack at N = 8 with the unpack on a CU-masked share of the chip (tools/probe_rank0.py)
set -u -o pipefail
source tools/gpu/outdir.sh r06 rank0
timeout -k 10 500 python -u tools/probe_rank0.py --n 8 --D 64 --root-ratio auto --cu-split 0,16,32,48,64 --it 6 > $O/rank0.jsonl 2>&1 || { tail -30 $O/rank0.jsonl; exit 1; }
cat $O/rank0.jsonl
