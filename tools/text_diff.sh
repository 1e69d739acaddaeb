#!/bin/bash
# Disassembly diff of one translation unit's gfx950 code object between two builds:
#   tools/text_diff.sh old.o new.o   -> the differing instruction lines (addresses stripped)
#   SORTED=1 tools/text_diff.sh ...  -> whether both hold the same instructions, only reordered
set -e -o pipefail
L=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
for k in 1 2; do
  o=$([ $k = 1 ] && echo "$1" || echo "$2")
  $L/llvm-objcopy -O binary --only-section=.hip_fatbin "$o" "$T/$k.fb"
  $L/clang-offload-bundler --unbundle --type=bc --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input="$T/$k.fb" --output="$T/$k.co"
  $L/llvm-objdump -d --no-show-raw-insn "$T/$k.co" | tail -n +4 | sed -E 's#[[:space:]]*//.*$##' > "$T/$k.s"
done
if [ "${SORTED:-0}" = 1 ]; then
  # the same instructions in another order: compare each side's sorted multiset of instruction lines
  sort "$T/1.s" > "$T/1.srt"; sort "$T/2.s" > "$T/2.srt"
  if cmp -s "$T/1.srt" "$T/2.srt"; then echo "same instruction multiset ($(wc -l < "$T/1.s") lines), $(diff "$T/1.s" "$T/2.s" | grep -c '^<') lines moved"; else echo "instruction multisets differ"; diff "$T/1.srt" "$T/2.srt" | head -20; fi
else
  diff "$T/1.s" "$T/2.s" || true
fi
rm -rf "$T"
