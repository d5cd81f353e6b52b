# LNW_PROF=1 per-workgroup timeline of one bench workload (phase means, grid
# timeline percentiles, per-XCC / per-CU spread), then the same workload timed
#   bash tools/gpu/timeline.sh TAG "BENCH ARGS"
set -o pipefail
TAG=$1; ARGS=$2
mkdir -p gpurun_out
LNW_PROF=1 timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 2 --warmup 5 $ARGS > gpurun_out/${TAG}_p.json 2> gpurun_out/${TAG}_p.err || exit 1
grep "lnw prof" gpurun_out/${TAG}_p.err | tail -14
timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 $ARGS > gpurun_out/${TAG}.json 2>/dev/null || exit 2
python -c "import json; d=json.load(open('gpurun_out/${TAG}.json')); print('$TAG', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
