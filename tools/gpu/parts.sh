# phase-S part timers: melee (contact variant, LNW_PROF) and config 4 with the
# group kernel's section timers (liblnw_prof.so built with -DLNW_GROUP_PROF)
set -o pipefail
mkdir -p gpurun_out
LNW_PROF=1 timeout -k 10 300 python bench.py --steps 3 --warmup 5 --no-cpu-baseline --no-secondary --spawns melee > gpurun_out/pm.json 2> gpurun_out/pm.err || exit 1
grep "lnw prof" gpurun_out/pm.err | tail -8
timeout -k 10 300 python bench.py --workload config4 --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 2
python -c "import json; d=json.load(open('gpurun_out/c4.json')); print('C4', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
LNW_LIB=$PWD/littoral-naval-warfare-marl_amd/lnw/liblnw_prof.so LNW_PROF=1 timeout -k 10 300 python bench.py --workload config4 --steps 3 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/c4p.json 2> gpurun_out/c4p.err || exit 3
grep "lnw prof" gpurun_out/c4p.err | tail -8
