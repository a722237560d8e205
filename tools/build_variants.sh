#!/bin/bash
# Build the measurement library convolutionalencdec_amd/lib/exp/measure/libviterbi_amd.so:
# the shipped sources with -DVTB_MEASURE, which honours the VTB_DEBUG bits that skip or
# corrupt output (bit 0: no traceback, 1: no ACS, 2: no traceback verification, 3: warm-up
# walk only, 4: return at entry) for phase timing.  The shipped library ignores those bits
# (vtb_api.hip read_knobs).  Load it with VTB_LIB_PATH=<dir>/libviterbi_amd.so; never ship it.
set -e
cd "$(dirname "$0")/.."
CS=convolutionalencdec_amd/csrc
d=convolutionalencdec_amd/lib/exp/measure; mkdir -p $d
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude -I$CS -DVTB_MEASURE "$@" \
    -o $d/libviterbi_amd.so $CS/vtb_api.hip $CS/vtb_lds_path.hip $CS/vtb_k7_lds.hip $CS/vtb_k9.hip $CS/vtb_gen.hip \
    $CS/vtb_genk.hip $CS/vtb_legacy.hip $CS/vtb_stream_gen.hip
