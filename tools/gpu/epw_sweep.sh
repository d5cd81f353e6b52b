# envs-per-workgroup sweep at small E (config 2 / config 3's per-GPU shard)
set -o pipefail
mkdir -p gpurun_out
for E in 8192 4096; do
  for EPW in 64 32 16 8; do
    LNW_EPW_RT=$EPW timeout -k 10 120 python bench.py --global-envs $E --no-secondary --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/epw_${E}_${EPW}.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/epw_${E}_${EPW}.json'));print($E,$EPW,round(d['ms_per_step']*1e3,1),'us/step',round(d['roofline']['kernel_ms_mean']*1e3,1),'us kernel')"
  done
done
