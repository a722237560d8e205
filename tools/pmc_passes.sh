#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, kernel trace only, no other tracing) for the
# workloads named on the command line, the library's sha written beside each workload's passes;
# summarise afterwards with
#   python tools/traffic_summary.py gpurun_out/pmc_<wl> r05 <key>
# Workloads (bench.py arguments, workload key):
#   head   K7 soft 4096 x 1024   (the bench line)      K7_soft_F4096_L1024   fetch write valu
#   c2     K7 hard 4096 x 1024                          K7_hard_F4096_L1024   fetch write valu
#   c3s    K7 soft 65536 x 2048                         K7_soft_F65536_L2048  fetch write valu
#   c3h    K7 hard 65536 x 2048                         K7_hard_F65536_L2048  fetch write valu
#   c4     K9 hard 4096 x 1024                          K9_hard_F4096_L1024   fetch write valu
#   c5     K7 soft 131072 x 1024 (C5's per-GPU shard)   K7_soft_F131072_L1024 fetch write valu
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
sha=$(sha256sum convolutionalencdec_amd/lib/libviterbi_amd.so | cut -c1-16)
for wl in "$@"; do
  passes="fetch write"
  case $wl in
    head) args="--steps 20 --warmup 2" ; passes="fetch write valu" ;;
    c2) args="--steps 20 --warmup 2 --hard" ; passes="fetch write valu" ;;
    c3s) args="--frames 65536 --frame-bits 2048 --steps 5 --warmup 1" ; passes="fetch write valu" ;;
    c3h) args="--frames 65536 --frame-bits 2048 --steps 5 --warmup 1 --hard" ; passes="fetch write valu" ;;
    c4) args="--K 9 --hard --steps 20 --warmup 2" ; passes="fetch write valu" ;;
    c5) args="--frames 131072 --steps 5 --warmup 1" ; passes="fetch write valu" ;;
    *) echo "unknown workload $wl"; exit 2 ;;
  esac
  mkdir -p gpurun_out/pmc_$wl && echo "$sha" > gpurun_out/pmc_$wl/lib_sha16.txt
  for pass in $passes; do
    case $pass in
      fetch) ctr="FETCH_SIZE" ;;
      write) ctr="WRITE_SIZE" ;;
      valu) ctr="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" ;;
    esac
    rm -rf gpurun_out/pmc_$wl/pmc_$pass
    timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/pmc_$wl/pmc_$pass -o run -- python3 bench.py $args --cpu-seconds 0 > gpurun_out/pmc_${wl}_$pass.log 2>&1 || { tail -5 gpurun_out/pmc_${wl}_$pass.log; exit 1; }
  done
  echo "pmc $wl done"
done
