# Kernel time of bench workloads under LNW_DEBUG_SKIP values of the diagnostics
# build (section skips: results change, timing attribution only):
#   bash tools/gpu/skip_ab.sh "BENCH ARGS" bits...
set -o pipefail
mkdir -p gpurun_out
ARGS=$1; shift
export LNW_LIB=$PWD/littoral-naval-warfare-marl_amd/lnw/liblnw_diag.so
for b in "$@"; do
  LNW_DEBUG_SKIP=$b timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 100 --warmup 10 $ARGS \
    > gpurun_out/skip.json 2>gpurun_out/skip.err || { tail -15 gpurun_out/skip.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/skip.json')); print('skip $b', '$ARGS', round(d['roofline']['kernel_ms_mean']*1e3, 1), 'us')"
done
