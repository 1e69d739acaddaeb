#!/bin/bash
# A variant of libbh_render.so whose bloom TU takes extra flags (the other TUs: the in-tree objects)
# usage: tools/build_bloom_variant.sh NAME "extra bloom-TU flags"
set -e
cd "$(dirname "$0")/.."
NAME=$1; EXTRA=$2
OUT=tools/variants/$NAME; mkdir -p $OUT
B=black_hole_ray_marching_amd/_build
hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-function -ffp-contract=off -fno-slp-vectorize \
  -mllvm -enable-post-misched=0 -mllvm -pragma-unroll-threshold=200000 $EXTRA -c black_hole_ray_marching_amd/csrc/bh_bloom.hip -o $OUT/b.o
hipcc -shared --offload-arch=gfx950 -o tools/variants/$NAME.so $(ls $B/*.o | grep -v bh_bloom.o) $OUT/b.o
echo tools/variants/$NAME.so
