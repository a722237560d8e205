#!/bin/bash
# Generic-kernel GPU step (measurement + parity): the generic families' GPU tests, gen_seg phase
# times, the batch sweep, the drop-in speedDecode protocol and (optional) a stream A/B against
# $STREAM_OLD_LIB.  Writes under gpurun_out/${ROUND:-r06}/generic_${TAG}.
#   usage: TAG=name bash tools/generic_check.sh [tests|time|sweep|speed|stream ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${ROUND:-r06}/generic_${TAG:-x}
mkdir -p "$O"
steps=${*:-tests time sweep speed}
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stream_gen.py \
        tests/test_gpu_lengths.py tests/test_gpu_tb_guard.py tests/test_gpu_frame_sync.py tests/test_gpu_parity.py \
        -m gpu > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
      tail -1 "$O/tests.log" ;;
    time)
      timeout -k 10 120 python -u tools/tstamp_seg.py > "$O/tstamp_seg.jsonl" 2> "$O/tstamp_seg.err" || exit 1
      cat "$O/tstamp_seg.jsonl" ;;
    sweep)
      timeout -k 10 300 python -u tools/generic_sweep.py --K 3,4,5,6,8 --L 1024,4096,16384 --rounds 1 \
        > "$O/sweep.jsonl" 2> "$O/sweep.err" || exit 1
      cut -c1-120 "$O/sweep.jsonl" ;;
    speed)
      timeout -k 10 200 python -u tools/legacy_speed.py --seconds 1 2>/dev/null | grep config > "$O/legacy_speed.jsonl" || exit 1
      cat "$O/legacy_speed.jsonl" ;;
    stream)
      : > "$O/stream_ab.txt"
      for r in 1 2; do
        for K in 3 5 6 8; do
          for lib in shipped ${STREAM_OLD_LIB:-}; do
            if [ "$lib" = shipped ]; then unset VTB_LIB_PATH; else export VTB_LIB_PATH=$lib; fi
            v=$(timeout -k 10 120 python bench.py --K $K --stream-chunk 1008 --steps 30 --warmup 3 --cpu-seconds 0 2>/dev/null \
                | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,1), round(d['value'],2), d['unit'])") || exit 1
            echo "r=$r K=$K lib=$lib us_per_call value unit: $v" | tee -a "$O/stream_ab.txt"
          done
        done
      done
      unset VTB_LIB_PATH ;;
  esac
done
