set -o pipefail
mkdir -p gpurun_out
for k in 0 1 1024; do
LNW_DEBUG_SKIP=$k timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bx.json 2> gpurun_out/bx.err || exit 4
python -c "import json; d=json.load(open('gpurun_out/bx.json')); print('skip=$k', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
done
