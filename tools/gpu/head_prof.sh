# headline timeline (LNW_PROF=1): workgroup start / stream start / wave-1 end
# spreads and the quiet-path phase means, plus the timed headline line
set -o pipefail
mkdir -p gpurun_out
LNW_PROF=1 timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 3 --warmup 5 > gpurun_out/hp.json 2> gpurun_out/hp.err || exit 1
grep "lnw prof" gpurun_out/hp.err | tail -11
timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/h.json 2>/dev/null || exit 2
python -c "import json; d=json.load(open('gpurun_out/h.json')); print('HEAD', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
