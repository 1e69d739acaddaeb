#!/bin/bash
# Round-2 GPU call B: lone-chain floor and frames-in-flight probes.
set -u
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 300 python -u tools/probe_chain.py > $O/probe_chain.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/probe_inflight.py > $O/probe_inflight.log 2>&1 || exit 12
echo done
