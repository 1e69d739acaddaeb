#!/bin/bash
# round 5: r05b (bloom wave phases + per-kernel roofline inputs) then r05c (shard per-tile cost probes)
set -u
tools/gpu/r05b.sh && tools/gpu/r05c.sh
