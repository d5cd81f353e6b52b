# headline kernel time vs envs per workgroup (LNW_EPW_RT): more, smaller
# workgroups than resident slots let finished CUs pick up new ones
set -o pipefail
mkdir -p gpurun_out
for EPW in 64 32 16 64; do
  LNW_EPW_RT=$EPW timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/he_$EPW.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/he_$EPW.json'));print('epw',$EPW,round(d['roofline']['kernel_ms_mean']*1e3,2),'us kernel')"
done
LNW_EPW_RT=32 LNW_PROF=1 timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 3 --warmup 5 2>&1 >/dev/null | grep "timeline\|quiet work" 
