#!/bin/bash
# Build measurement-only variants of libviterbi_amd.so into convolutionalencdec_amd/lib/exp/<name>/.
set -e
cd "$(dirname "$0")/.."
CS=convolutionalencdec_amd/csrc
build() {
  name=$1; shift
  d=convolutionalencdec_amd/lib/exp/$name; mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude -I$CS "$@" \
      -o $d/libviterbi_amd.so $CS/vtb_api.hip $CS/vtb_lds_path.hip $CS/vtb_reg_path.hip
}
for v in "$@"; do
  case $v in
    nostore) build nostore -DVTB_EXP_NO_STORE ;;
    nodecide) build nodecide -DVTB_EXP_NO_DECIDE ;;
    noexch) build noexch -DVTB_EXP_NO_EXCHANGE ;;
    bare) build bare -DVTB_EXP_NO_DECIDE -DVTB_EXP_NO_EXCHANGE ;;
    warm96) build warm96 -DVTB_WARM=96 ;;
    warm144) build warm144 -DVTB_WARM=144 ;;
    *) echo "unknown variant $v"; exit 1 ;;
  esac
done
