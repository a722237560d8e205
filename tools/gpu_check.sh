set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m3 -E 'gfx|Marketing' > gpurun_out/devinfo.txt || true
nproc > gpurun_out/nproc.txt
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || exit $?
