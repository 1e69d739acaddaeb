#!/bin/bash
# Dump the gfx950 assembly of the exact (or fast) march TU with extra flags:
#   tools/isa.sh NAME exact|fast "extra flags"   -> /tmp/isa_NAME/*.s
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
NAME=$1; MODE=$2; EXTRA=$3
D=/tmp/isa_$NAME; mkdir -p $D; cd $D
C="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-function --save-temps"
if [ "$MODE" = fast ]; then F="-ffp-contract=fast -fno-hip-fp32-correctly-rounded-divide-sqrt"
else F="-ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize ${SCHED--mllvm -enable-misched=0 -mllvm -enable-post-misched=0}"; fi
hipcc $C $F $EXTRA -c $R/black_hole_ray_marching_amd/csrc/bh_march_$MODE.hip -o $D/x.o 2>/dev/null
ls $D/*gfx950*.s
