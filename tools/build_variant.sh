#!/bin/bash
# Build a variant of libbh_render.so with extra flags for the exact TU into tools/variants/NAME.so
# usage: tools/build_variant.sh NAME "extra exact-TU flags"
set -e
cd "$(dirname "$0")/.."
NAME=$1; EXTRA=$2
OUT=tools/variants/$NAME; mkdir -p $OUT
C="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-function"
S=black_hole_ray_marching_amd/csrc
hipcc $C -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize ${SCHED--mllvm -enable-misched=0 -mllvm -enable-post-misched=0 -mllvm -disable-machine-licm} $EXTRA -c $S/bh_march_exact.hip -o $OUT/e.o
hipcc $C -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize ${LAT_EXTRA-$EXTRA} -c $S/bh_march_exact_lat.hip -o $OUT/el.o
hipcc $C -ffp-contract=fast -fno-hip-fp32-correctly-rounded-divide-sqrt ${FAST_EXTRA--mllvm -enable-misched=0 -mllvm -enable-post-misched=0} -c $S/bh_march_fast.hip -o $OUT/f.o
hipcc $C -c $S/bh_tiles.hip -o $OUT/t.o
hipcc $C -ffp-contract=off ${BLOOM_EXTRA--fno-slp-vectorize -mllvm -enable-post-misched=0 -mllvm -pragma-unroll-threshold=200000} -c $S/bh_bloom.hip -o $OUT/b.o
hipcc $C -ffp-contract=off -c $S/bh_selftest.hip -o $OUT/s.o
hipcc $C -ffp-contract=off -x hip -c $S/bh_host.cpp -o $OUT/h.o
hipcc -shared --offload-arch=gfx950 -o tools/variants/$NAME.so $OUT/*.o
echo tools/variants/$NAME.so
