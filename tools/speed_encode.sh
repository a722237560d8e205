#!/bin/bash
# The reference's speedEncode harness (pinned to CPU 16 by its source) on the GPU box's host,
# against the reference's encoder and against the drop-in's; a few seconds each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
secs=${1:-5}
for b in ref amd; do
  oracle/_ref/speedEncode_$b > gpurun_out/speedEncode_$b.log 2>&1 &
  pid=$!; sleep $secs; kill $pid; wait $pid 2>/dev/null
  grep -h "Rate" gpurun_out/speedEncode_$b.log | grep -v "Rate: 0.5" | tail -3 | sed "s/^/$b: /"
done
exit 0
