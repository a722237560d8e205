set -o pipefail
mkdir -p gpurun_out/r04
echo "== round-3 library" 
VTB_LIB_PATH=$PWD/convolutionalencdec_amd/lib/exp/libviterbi_amd_r03.so timeout -k 10 300 python -u tools/dbg_frame_case.py --i 1366 --L 2966 --noise 0.5 > gpurun_out/r04/dbg_case1366_r03lib.txt 2>&1 || exit $?
echo "== fixed library"
timeout -k 10 300 python -u tools/dbg_frame_case.py --i 1366 --L 2966 --noise 0.5 > gpurun_out/r04/dbg_case1366_fixed.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_split_fixup.py -x -v -k case_1366 --timeout 300 --timeout-method thread > gpurun_out/r04/case1366_tests.log 2>&1
[ $? -eq 0 ] || exit 1
bash tools/gpu_r04.sh gputests smoke bench prof || exit 1
# K=9 C4: what the survivor stores cost the ACS (no traceback: VTB_DEBUG=1), base vs no stores
E=convolutionalencdec_amd/lib/exp
VARIANTS="$E/base $E/k9noword" VTB_DEBUG=1 bash tools/ab_variants.sh 3 --K 9 --hard && cp gpurun_out/ab.txt gpurun_out/r04/ab_k9noword_acs_only.txt || exit 1
# headline: staging writes of lanes 48-63 masked off (LDS bank conflicts)
VARIANTS="$E/base $E/stage48" bash tools/ab_variants.sh 4 && cp gpurun_out/ab.txt gpurun_out/r04/ab_stage48.txt
