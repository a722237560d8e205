set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/gws_breakdown.txt; : > $out
for d in 0 1 3; do
  r=$(VTB_KERNEL=gws VTB_DEBUG=$d timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms']*1000)") || exit 1
  echo "gws dbg=$d kernel_us=$r" | tee -a $out
done
for C in 1008 4080; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 3 --cpu-seconds 0 --stream-chunk $C 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('stream C=$C', d['ms_per_step']*1000, d['value'])" | tee -a $out || exit 1
done
