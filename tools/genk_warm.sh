# Measurement only: the general-k decoder's time against its traceback warm-up
# ($VTB_GENK_WARM, exact for any value: the block walks are verified).  Usage: genk_warm.sh W...
mkdir -p gpurun_out/r03
export FRAMES=${FRAMES:-16384}
for w in "$@"; do
  echo "warm $w"
  VTB_GENK_WARM=$w timeout -k 10 200 python3 tools/genk_scale.py || exit 1
done > gpurun_out/r03/genk_warm.jsonl 2>&1
