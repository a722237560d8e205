#!/bin/bash
# Per-kernel VGPR / SGPR / spill / LDS figures of the gfx950 code object inside a hipcc-built
# .o (the AMDGPU metadata note), one line per kernel:  name vgpr sgpr spill_v spill_s lds
#   usage: tools/kernel_resources.sh file.o
set -euo pipefail
B=/opt/rocm/lib/llvm/bin
t=$(mktemp -d)
trap 'rm -rf "$t"' EXIT
"$B/llvm-objcopy" --dump-section=.hip_fatbin="$t/fb" "$1"
"$B/clang-offload-bundler" --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input="$t/fb" --output="$t/co" --unbundle
"$B/llvm-readelf" --notes "$t/co" | python3 -c '
import sys, re
txt = sys.stdin.read()
for blk in re.split(r"\n\s*- \.agpr_count", txt)[1:]:
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    print(g("name"), "vgpr", g("vgpr_count"), "sgpr", g("sgpr_count"), "spill_v", g("vgpr_spill_count"),
          "spill_s", g("sgpr_spill_count"), "lds", g("group_segment_fixed_size"))
'
