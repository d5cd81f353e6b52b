# melee (contact variant) LNW_PROF timeline and SIMD-placement diagnostics, then the timed melee line
set -o pipefail
mkdir -p gpurun_out
LNW_PROF=1 timeout -k 10 120 python bench.py --steps 3 --warmup 5 --no-cpu-baseline --no-secondary --spawns melee > gpurun_out/pm.json 2> gpurun_out/pm.err || exit 1
grep "lnw prof" gpurun_out/pm.err | grep -v "per agent\|parts" | tail -9
timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-secondary --spawns melee > gpurun_out/bm.json 2> gpurun_out/bm.err || exit 2
python -c "import json; d=json.load(open('gpurun_out/bm.json')); print('MELEE', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
