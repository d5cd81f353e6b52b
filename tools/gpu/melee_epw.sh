# melee kernel time vs envs per workgroup (LNW_EPW_RT): smaller workgroups,
# less SIMT divergence per wave, more of them than resident slots
set -o pipefail
mkdir -p gpurun_out
for EPW in 64 32 16; do
  LNW_EPW_RT=$EPW timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 100 --warmup 10 --spawns melee > gpurun_out/me_$EPW.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/me_$EPW.json'));print('melee epw',$EPW,round(d['roofline']['kernel_ms_mean']*1e3,2),'us kernel')"
done
