#!/bin/bash
# Disassemble the gfx950 code object inside a hipcc-built .o (its .hip_fatbin bundle) to
# stdout, addresses stripped, so two builds can be compared with diff: a source cleanup that
# must not change the kernels (e.g. removing closed VTB_EXP_* experiments) is checked by an
# empty diff.   usage: tools/isa_dump.sh file.o > file.s
set -euo pipefail
B=/opt/rocm/lib/llvm/bin
o=$1
t=$(mktemp -d)
trap 'rm -rf "$t"' EXIT
"$B/llvm-objcopy" --dump-section=.hip_fatbin="$t/fb" "$o"
"$B/clang-offload-bundler" --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input="$t/fb" --output="$t/co" --unbundle
"$B/llvm-objdump" -d --no-show-raw-insn --no-leading-addr "$t/co" | tail -n +3 | sed -e 's/ *\/\/ [0-9A-F]*:.*$//' -e 's/<[^>]*+0x[0-9a-f]*>//'
