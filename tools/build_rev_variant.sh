#!/bin/bash
# Build libbh_render.so of another git revision (its csrc/ and include/) into tools/variants/NAME.so, with
# the product's per-TU flags: A/B of the working tree against a committed version.
#   tools/build_rev_variant.sh NAME REV
set -e
cd "$(dirname "$0")/.."
NAME=$1; REV=$2
T=/tmp/bh_rev_$NAME; rm -rf $T; mkdir -p $T/black_hole_ray_marching_amd/csrc $T/include
for f in $(git ls-tree --name-only $REV black_hole_ray_marching_amd/csrc/); do git show $REV:$f > $T/$f; done
git show $REV:include/bh_render.h > $T/include/bh_render.h
OUT=tools/variants/$NAME; mkdir -p $OUT
C="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-function"
S=$T/black_hole_ray_marching_amd/csrc
hipcc $C -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -mllvm -enable-misched=0 -mllvm -enable-post-misched=0 -mllvm -disable-machine-licm -c $S/bh_march_exact.hip -o $OUT/e.o
hipcc $C -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -c $S/bh_march_exact_lat.hip -o $OUT/el.o
hipcc $C -ffp-contract=fast -fno-hip-fp32-correctly-rounded-divide-sqrt -mllvm -enable-misched=0 -mllvm -enable-post-misched=0 -c $S/bh_march_fast.hip -o $OUT/f.o
hipcc $C -c $S/bh_tiles.hip -o $OUT/t.o
hipcc $C -ffp-contract=off -fno-slp-vectorize -mllvm -enable-post-misched=0 -c $S/bh_bloom.hip -o $OUT/b.o
hipcc $C -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -c $S/bh_selftest.hip -o $OUT/s.o
hipcc $C -ffp-contract=off -x hip -c $S/bh_host.cpp -o $OUT/h.o
hipcc -shared --offload-arch=gfx950 -o tools/variants/$NAME.so $OUT/*.o
rm -rf $OUT $T
echo tools/variants/$NAME.so
