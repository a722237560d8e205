set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/isa_bench2 tools/probes/isa_bench2.hip && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/isa_bench3 tools/probes/isa_bench3.hip && timeout -k 10 120 /tmp/isa_bench2 > gpurun_out/isa_bench2.log 2>&1 && timeout -k 10 120 /tmp/isa_bench3 > gpurun_out/isa_bench3.log 2>&1
