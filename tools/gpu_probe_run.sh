set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ber.py -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ber.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --frames 65536 > gpurun_out/b65a.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 200 --warmup 3 --cpu-seconds 0 --frames 65536 > gpurun_out/b65b.log 2>&1 || exit $?
timeout -k 10 120 python tools/host_path_probe.py 4096 > gpurun_out/host4k.log 2>&1 || exit $?
timeout -k 10 120 python tools/host_path_probe.py 65536 > gpurun_out/host64k.log 2>&1 || exit $?
