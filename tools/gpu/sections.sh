# LNW_PROF=1 section timers of the diagnostics build (liblnw_diag.so: the
# group kernel's and the contact variant's per-section sums, slowest workgroup,
# phase-S spread) for bench workloads, then the production build timed:
#   bash tools/gpu/sections.sh TAG "BENCH ARGS" [TAG "BENCH ARGS" ...]
set -o pipefail
mkdir -p gpurun_out
DIAG=$PWD/littoral-naval-warfare-marl_amd/lnw/liblnw_diag.so
while [ $# -ge 2 ]; do
  TAG=$1; ARGS=$2; shift 2
  LNW_LIB=$DIAG LNW_PROF=1 timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 2 --warmup 10 $ARGS \
    > gpurun_out/${TAG}_sec.json 2> gpurun_out/${TAG}_sec.err || exit 1
  grep "lnw prof" gpurun_out/${TAG}_sec.err | tail -8
  timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 100 --warmup 10 $ARGS > gpurun_out/${TAG}.json 2>/dev/null || exit 2
  python -c "import json; d=json.load(open('gpurun_out/${TAG}.json')); print('$TAG', round(d['value']/1e6, 2), 'M', round(d['roofline']['kernel_ms_mean']*1e3, 1), 'us')"
done
