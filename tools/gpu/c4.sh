# config 4 (8 192 envs, 8v10 + 2 LS, 200x200): bench line and LNW_PROF phase timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload config4 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -20 gpurun_out/c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c4.json')); print('C4', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
LNW_PROF=1 timeout -k 10 300 python bench.py --workload config4 --steps 3 --warmup 5 --no-cpu-baseline > gpurun_out/c4p.json 2> gpurun_out/c4p.err || exit 2
grep "lnw prof" gpurun_out/c4p.err | tail -4
