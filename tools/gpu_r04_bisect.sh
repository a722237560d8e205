set -o pipefail
mkdir -p gpurun_out/r04
echo "== round-3 library" 
VTB_LIB_PATH=$PWD/convolutionalencdec_amd/lib/exp/libviterbi_amd_r03.so timeout -k 10 300 python -u tools/dbg_frame_case.py --i 1366 --L 2966 --noise 0.5 > gpurun_out/r04/dbg_case1366_r03lib.txt 2>&1 || exit $?
echo "== fixed library"
timeout -k 10 300 python -u tools/dbg_frame_case.py --i 1366 --L 2966 --noise 0.5 > gpurun_out/r04/dbg_case1366_fixed.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_split_fixup.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/split_fixup_tests.log 2>&1
