# kernel time of one bench workload with LNW_DEBUG_SKIP bit sets (diagnostics)
#   bash tools/gpu/skip_multi.sh "BENCH ARGS" BITS...
set -o pipefail
mkdir -p gpurun_out
ARGS=$1; shift
for bits in "$@"; do
  LNW_DEBUG_SKIP=$bits timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline --steps 40 --warmup 5 $ARGS > gpurun_out/sk.json 2> gpurun_out/sk.err || { tail -5 gpurun_out/sk.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sk.json'));print('$ARGS', 'bits $bits kernel us', round(d['roofline']['kernel_ms_mean']*1e3,1))"
done
