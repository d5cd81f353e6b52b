# quick A/B: default bench line twice, melee line and the LNW_PROF phase-S split
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/ab_ref$r.json 2> gpurun_out/ab_ref$r.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/ab_ref$r.json')); print('REF', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
done
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --spawns melee > gpurun_out/ab_m.json 2> gpurun_out/ab_m.err || exit 2
python -c "import json; d=json.load(open('gpurun_out/ab_m.json')); print('MELEE', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
LNW_PROF=1 timeout -k 10 300 python bench.py --steps 3 --warmup 5 --no-cpu-baseline --no-secondary --spawns melee > gpurun_out/ab_pm.json 2> gpurun_out/ab_pm.err || exit 3
grep "lnw prof" gpurun_out/ab_pm.err | tail -2
