#!/bin/bash
# Round 2: rocprofv3 PMC passes on the shipped library (FETCH_SIZE, WRITE_SIZE and the SQ VALU
# pass, each its own run, --kernel-trace only), per workload: the headline (K=7 soft 4096 x
# 1024), K=7 hard 4096 x 1024, and config C3 soft / hard (65,536 x 2,048).  Summarised (and
# stamped with the library hash) by tools/traffic_summary.py on the build host.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02pmc; mkdir -p $o
export TMPDIR=/tmp
for wl in K7_soft_F4096_L1024 K7_hard_F4096_L1024 K7_soft_F65536_L2048 K7_hard_F65536_L2048; do
  args="--steps 10 --warmup 2 --cpu-seconds 0"
  case $wl in *hard*) args="$args --hard" ;; esac
  case $wl in *F65536*) args="$args --frames 65536 --frame-bits 2048 --gen device" ;; esac
  for pass in fetch write valu; do
    case $pass in
      fetch) ctr="FETCH_SIZE" ;;
      write) ctr="WRITE_SIZE" ;;
      valu) ctr="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" ;;
    esac
    rm -rf $o/$wl/pmc_$pass
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $o/$wl/pmc_$pass -o run -- python3 bench.py $args > $o/${wl}_$pass.log 2>&1 || exit $?
  done
done
exit 0
