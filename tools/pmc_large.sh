#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 run each) for the large-batch workloads, for
# bench.py's roofline.traffic (tools/traffic_summary.py gpurun_out/pmc_<wl> r01 <key>).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in 65k 65k2048; do
  case $wl in
    65k) args="--frames 65536 --steps 5 --warmup 1 --cpu-seconds 0 --gen device" ;;
    65k2048) args="--frames 65536 --frame-bits 2048 --steps 5 --warmup 1 --cpu-seconds 0 --gen device" ;;
  esac
  for pass in fetch write; do
    case $pass in fetch) ctr=FETCH_SIZE ;; write) ctr=WRITE_SIZE ;; esac
    rm -rf gpurun_out/pmc_$wl/pmc_$pass
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/pmc_$wl/pmc_$pass -o run -- python3 bench.py $args > gpurun_out/pmc_${wl}_$pass.log 2>&1 || exit $?
  done
done
