#!/bin/bash
# Build measurement-only variants of libviterbi_amd.so into convolutionalencdec_amd/lib/exp/<name>/.
set -e
cd "$(dirname "$0")/.."
CS=convolutionalencdec_amd/csrc
build() {
  name=$1; shift
  d=convolutionalencdec_amd/lib/exp/$name; mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude -I$CS "$@" \
      -o $d/libviterbi_amd.so $CS/vtb_api.hip $CS/vtb_lds_path.hip $CS/vtb_k7_lds.hip $CS/vtb_k9.hip $CS/vtb_gen.hip $CS/vtb_genk.hip $CS/vtb_legacy.hip $CS/vtb_stream_gen.hip
}
for v in "$@"; do
  case $v in
    nostore) build nostore -DVTB_EXP_NO_STORE ;;
    nolds) build nolds -DVTB_EXP_NO_LDS ;;
    nocmp) build nocmp -DVTB_EXP_NO_CMP ;;
    nostore_nolds) build nostore_nolds -DVTB_EXP_NO_STORE -DVTB_EXP_NO_LDS ;;
    nostage) build nostage -DVTB_EXP_NO_STAGE ;;
    ahead3) build ahead3 -DVTB_EXP_AHEAD=3 ;;
    notabread) build notabread -DVTB_EXP_NO_TABREAD ;;
    notab) build notab -DVTB_EXP_NO_TABREAD -DVTB_EXP_NO_STAGE ;;
    rawnowait) build rawnowait -DVTB_EXP_RAWNOWAIT ;;
    warm96) build warm96 -DVTB_EXP_TBWARM=96 ;;
    warm144) build warm144 -DVTB_EXP_TBWARM=144 ;;
    noword) build noword -DVTB_EXP_NO_WORD ;;
    base) build base ;;
    k9ah3) build k9ah3 -DVTB_EXP_K9AH=3 -DVTB_EXP_K9RS=4 ;;
    wpe2) build wpe2 -DVTB_EXP_WPE=2 ;;
    wpe4) build wpe4 -DVTB_EXP_WPE=4 ;;
    k9ah5) build k9ah5 -DVTB_EXP_K9AH=5 -DVTB_EXP_K9RS=6 ;;
    noprio) build noprio -DVTB_EXP_NOPRIO ;;
    tbspec) build tbspec -DVTB_EXP_TBSPEC ;;
    nonop) build nonop -DVTB_EXP_NONOP ;;
    bitop3) build bitop3 -DVTB_EXP_BITOP3 ;;
    rd1) build rd1 -DVTB_EXP_RD1 ;;
    tab32) build tab32 -DVTB_EXP_TAB32 ;;
    swz16) build swz16 -DVTB_EXP_SWZ=1 ;;
    swz) build swz -DVTB_EXP_SWZ=2 ;;
    rn16) build rn16 -DVTB_EXP_RN=16 ;;
    nostage_noword) build nostage_noword -DVTB_EXP_NO_STAGE -DVTB_EXP_NO_WORD ;;
    e32) build e32 -DVTB_EXP_E32 ;;
    sgmask) build sgmask -DVTB_EXP_SGMASK ;;
    e32sg) build e32sg -DVTB_EXP_E32 -DVTB_EXP_SGMASK ;;
    b128) build b128 -DVTB_EXP_B128 ;;
    k9noword) build k9noword -DVTB_EXP_K9_NOWORD ;;
    stage48) build stage48 -DVTB_EXP_STAGE48 ;;
    k9nt) build k9nt -DVTB_EXP_K9_NT ;;
    k9noswap) build k9noswap -DVTB_EXP_K9_NOSWAP ;;
    prio*) build $v -DVTB_EXP_PRIO=${v#prio} ;;
    k9prio*) build $v -DVTB_EXP_K9PRIO=${v#k9prio} ;;
    *) echo "unknown variant $v"; exit 1 ;;
  esac
done
