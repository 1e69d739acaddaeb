#!/bin/bash
# Sourced by the round-5+ GPU scripts: O = a fresh output directory for THIS call,
# gpurun_out/<round>/<script>/<UTC time>-<pid>, so that a retry never overwrites the log of a failing run
# (VERDICT r4 item 1).  Usage: source tools/gpu/outdir.sh r05 name
R=${1:?round}; N=${2:?name}
O=gpurun_out/$R/$N/$(date -u +%Y%m%dT%H%M%S)-$$
if [ -e "$O" ]; then echo "refusing to reuse $O" >&2; exit 3; fi
mkdir -p "$O" || exit 3
echo "output: $O"
