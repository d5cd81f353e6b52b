# config 4 iteration: group-kernel parity tests, then the timed config-4 line and its LNW_PROF summary
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "group or config4" > gpurun_out/tc4.log 2>&1 || { tail -30 gpurun_out/tc4.log; exit 1; }
tail -2 gpurun_out/tc4.log
timeout -k 10 120 python bench.py --workload config4 --no-secondary --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/c4.json 2>/dev/null || exit 2
python -c "import json; d=json.load(open('gpurun_out/c4.json')); print('C4', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
LNW_PROF=1 timeout -k 10 120 python bench.py --workload config4 --steps 3 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/c4p.json 2> gpurun_out/c4p.err || exit 3
grep "group kernel LDS\|span per" gpurun_out/c4p.err | tail -2
