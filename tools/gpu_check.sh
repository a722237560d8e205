#!/bin/bash
# GPU-box check: parity tests, smoke, bench (+ optional rocprofv3 kernel-trace summary).
# Usage (through gpurun): bash tools/gpu_check.sh [tests] [smoke] [bench] [prof] [pmc]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
steps="${*:-tests smoke bench}"
export TMPDIR=/tmp
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
      rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
      [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $? ;;
    bench)
      timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || exit $?
      VTB_KERNEL=lds timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/bench_lds.log 2>&1 || exit $?
      timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --hard > gpurun_out/bench_hard.log 2>&1 || exit $?
      timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --frames 65536 > gpurun_out/bench_65k.log 2>&1 || exit $? ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/prof.log 2>&1 || exit $?
      rm -rf gpurun_out/prof_hard
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hard -o run -- python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 --hard > gpurun_out/prof_hard.log 2>&1 || exit $? ;;
    pmc)
      # per workload: FETCH_SIZE, WRITE_SIZE and the SQ VALU pass, each its own rocprofv3 run
      for wl in soft hard; do
        args="--steps 20 --warmup 2 --cpu-seconds 0"; [ $wl = hard ] && args="$args --hard"
        for pass in fetch write valu; do
          case $pass in
            fetch) ctr="FETCH_SIZE" ;;
            write) ctr="WRITE_SIZE" ;;
            valu) ctr="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" ;;
          esac
          rm -rf gpurun_out/pmc_${wl}/pmc_$pass
          timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/pmc_${wl}/pmc_$pass -o run -- python3 bench.py $args > gpurun_out/pmc_${wl}_$pass.log 2>&1 || exit $?
        done
      done ;;
    isa)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/isa_bench tools/probes/isa_bench.hip &&
      timeout -k 10 120 /tmp/isa_bench > gpurun_out/isa_bench.log 2>&1 || exit $? ;;
  esac
done
exit 0
