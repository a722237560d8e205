#!/bin/bash
# Round 3 GPU steps, each under its own time limit, stopping at the first failure:
#   bash tools/gpu_r03.sh tests:<pytest args> | bench | prof | peer | strong | smoke ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03; mkdir -p $o
export TMPDIR=/tmp
for s in "$@"; do
  case $s in
    tests:*) t="${s#tests:}"; n=$(echo "$t" | tr -c 'a-zA-Z0-9_' '_' | cut -c1-60)
             timeout -k 10 900 python3 -u -m pytest $t -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
               > $o/tests_$n.log 2>&1 || { tail -40 $o/tests_$n.log; exit 1; } ; tail -3 $o/tests_$n.log ;;
    gputests) timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
               > $o/gpu_tests_full.log 2>&1 || { tail -40 $o/gpu_tests_full.log; exit 1; } ; tail -3 $o/gpu_tests_full.log ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { cat $o/smoke.log; exit 1; } ;;
    bench) timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
           cat $o/bench.json ;;
    bench50) timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 5 --cpu-seconds 0 > $o/bench50.json 2> $o/bench50.err || exit 1
           cat $o/bench50.json ;;
    prof) rm -rf $o/prof
          timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $o/prof.json 2> $o/prof.err || { tail $o/prof.err; exit 1; } ;;
    peer) timeout -k 10 300 python3 bench.py --gpus 1 --source gpu0 --peer-devices 0,0 --peer-stage-all --global-frames 131072 --steps 5 --warmup 2 > $o/peer_rehearsal.json 2> $o/peer.err || { tail $o/peer.err; exit 1; }
          cat $o/peer_rehearsal.json ;;
    strong) timeout -k 10 300 python3 bench.py --gpus 1 --global-frames 131072 --steps 10 --warmup 3 --cpu-seconds 0 > $o/strong_c5_shard.json 2> $o/strong.err || { tail $o/strong.err; exit 1; }
          cat $o/strong_c5_shard.json ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
