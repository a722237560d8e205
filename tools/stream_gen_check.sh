set -o pipefail
mkdir -p gpurun_out/r06/strm2
PYT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT -x tests/test_gpu_stream_gen.py tests/test_gpu_tb_guard.py tests/test_gpu_stream.py -m gpu > gpurun_out/r06/strm2/tests.log 2>&1 || { tail -30 gpurun_out/r06/strm2/tests.log; exit 1; }
tail -1 gpurun_out/r06/strm2/tests.log
VTB_FUZZ_N=2000 VTB_FUZZ_SEED=6605 timeout -k 10 600 $PYT tests/test_gpu_fuzz.py -m gpu -k stream_random > gpurun_out/r06/strm2/fuzz_stream.log 2>&1 || { tail -30 gpurun_out/r06/strm2/fuzz_stream.log; exit 1; }
tail -1 gpurun_out/r06/strm2/fuzz_stream.log
VTB_DEBUG=131072 VTB_FUZZ_N=600 VTB_FUZZ_SEED=6606 timeout -k 10 600 $PYT tests/test_gpu_fuzz.py -m gpu -k stream_random > gpurun_out/r06/strm2/fuzz_stream_forced.log 2>&1 || { tail -30 gpurun_out/r06/strm2/fuzz_stream_forced.log; exit 1; }
tail -1 gpurun_out/r06/strm2/fuzz_stream_forced.log
for F in 4096 32768; do for K in 3 4 5 6 8; do
  timeout -k 10 120 python bench.py --K $K --frames $F --stream-chunk 1008 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/r06/strm2/s_${K}_${F}.json 2> gpurun_out/r06/strm2/s_${K}_${F}.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value']/1000,2), d['ms_per_step'])" gpurun_out/r06/strm2/s_${K}_${F}.json $K $F
done; done
