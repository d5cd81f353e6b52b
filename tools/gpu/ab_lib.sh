# Interleaved A/B of two builds (kernel time per step):
#   bash tools/gpu/ab_lib.sh ROUNDS LIB_A LIB_B "BENCH ARGS" ["BENCH ARGS" ...]
set -o pipefail
mkdir -p gpurun_out
R=$1; A=$2; B=$3; shift 3
for r in $(seq "$R"); do
  for args in "$@"; do
    for lib in "$A" "$B"; do
      LNW_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 $args \
        > gpurun_out/ab.json 2>/dev/null || exit 1
      python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('r$r', '$(basename $lib)', '$args', round(d['roofline']['kernel_ms_mean']*1e3, 2), 'us')"
    done
  done
done
