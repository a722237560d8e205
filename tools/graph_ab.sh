set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/graph_ab.txt
for i in 1 2; do
for g in "" "--graph"; do
  for wl in "" "--hard"; do
    r=$(timeout -k 10 120 python bench.py --steps 100 --warmup 5 --cpu-seconds 0 $g $wl 2>gpurun_out/graph_err.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, d['roofline']['kernel_ms']*1000, d['value'])") || exit 1
    echo "graph=$g wl=$wl step_us,kernel_us,value=$r" | tee -a gpurun_out/graph_ab.txt
  done
done
done
