#!/bin/bash
# The reference's speedDecode harness, unchanged, on the GPU box (oracle/Makefile `harness`):
# first built against the reference library (CPU), then against the legacy drop-in
# (include/viterbiDecoder.h -> libviterbi_legacy_k7 -> GPU, one frame per call).  The harness
# loops forever printing a rate per second; each run is stopped after a few seconds.  The
# GPU-using run is the last step of the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
secs=${1:-6}
oracle/_ref/speedDecode_ref > gpurun_out/speedDecode_ref.log 2>&1 &
pid=$!; sleep $secs; kill $pid; wait $pid 2>/dev/null
oracle/_ref/speedDecode_amd > gpurun_out/speedDecode_amd.log 2>&1 &
pid=$!; sleep $((secs + 4)); kill $pid; wait $pid 2>/dev/null
grep -h "Rate" gpurun_out/speedDecode_ref.log | tail -3 | sed 's/^/ref: /'
grep -h "Rate" gpurun_out/speedDecode_amd.log | tail -3 | sed 's/^/amd: /'
if [ "$2" = k9 ]; then  # the K=9 configuration (params/k9)
  oracle/_ref/speedDecode_ref_k9 > gpurun_out/speedDecode_ref_k9.log 2>&1 &
  pid=$!; sleep $secs; kill $pid; wait $pid 2>/dev/null
  oracle/_ref/speedDecode_amd_k9 > gpurun_out/speedDecode_amd_k9.log 2>&1 &
  pid=$!; sleep $((secs + 4)); kill $pid; wait $pid 2>/dev/null
  grep -h "Rate" gpurun_out/speedDecode_ref_k9.log | tail -3 | sed 's/^/ref K=9: /'
  grep -h "Rate" gpurun_out/speedDecode_amd_k9.log | tail -3 | sed 's/^/amd K=9: /'
fi
if [ -n "$HARNESS_ALL" ]; then  # every other configuration the drop-in builds (params/<cfg>)
  for c in k3s k4 k5 k6 k8; do
    oracle/_ref/speedDecode_ref_$c > gpurun_out/speedDecode_ref_$c.log 2>&1 &
    pid=$!; sleep $secs; kill $pid; wait $pid 2>/dev/null
    oracle/_ref/speedDecode_amd_$c > gpurun_out/speedDecode_amd_$c.log 2>&1 &
    pid=$!; sleep $((secs + 4)); kill $pid; wait $pid 2>/dev/null
    grep -h "Rate" gpurun_out/speedDecode_ref_$c.log | tail -3 | sed "s/^/ref $c: /"
    grep -h "Rate" gpurun_out/speedDecode_amd_$c.log | tail -3 | sed "s/^/amd $c: /"
  done
fi
exit 0
