#!/bin/bash
# sha256 of the gfx950 .text of every translation unit's device code object (black_hole_ray_marching_amd/_build/*.o):
# identical hashes before and after a source edit prove the edit left the shipped kernels' machine code unchanged.
#   tools/text_hash.sh [build_dir]
set -e -o pipefail
B=${1:-"$(cd "$(dirname "$0")/.." && pwd)/black_hole_ray_marching_amd/_build"}
L=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
for o in "$B"/*.o; do
  n=$(basename "$o" .o)
  $L/llvm-objcopy -O binary --only-section=.hip_fatbin "$o" "$T/$n.fb"
  [ -s "$T/$n.fb" ] || continue
  $L/clang-offload-bundler --unbundle --type=bc --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input="$T/$n.fb" --output="$T/$n.co"
  $L/llvm-objcopy -O binary --only-section=.text "$T/$n.co" "$T/$n.text"
  echo "$(sha256sum < "$T/$n.text" | cut -c1-16) $(stat -c %s "$T/$n.text") $n"
done
rm -rf "$T"
