# kernel time with sections disabled (LNW_DEBUG_SKIP bits; results differ, timing only):
# 128 get_obs, 65536 fire, 8192 walk, 16384 bearings+fixes, 131072 fixes,
# 262144 gauss draws, 524288 tan, 32768 LOS loads, 1048576 target-list stores
#   bash tools/gpu/c4_skip.sh "<bench args>" bit...
set -o pipefail
mkdir -p gpurun_out
ARGS=$1; shift
for B in 0 "$@"; do
  LNW_DEBUG_SKIP=$B timeout -k 10 120 python bench.py $ARGS --no-secondary --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/sk_$B.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sk_$B.json'));print('skip',$B,round(d['roofline']['kernel_ms_mean']*1e3,1),'us kernel')"
done
