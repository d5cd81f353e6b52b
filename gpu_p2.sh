set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tgpu.log 2>&1 || { tail -30 gpurun_out/tgpu.log; exit 1; }
tail -1 gpurun_out/tgpu.log
for k in 0 4096; do
LNW_DEBUG_SKIP=$k timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --workload config4 > gpurun_out/b4.json 2> gpurun_out/b4.err || exit 6
python -c "import json; d=json.load(open('gpurun_out/b4.json')); print('CFG4 skip=$k', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
done
