set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tgpu.log 2>&1 || { tail -30 gpurun_out/tgpu.log; exit 1; }
tail -2 gpurun_out/tgpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 3
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('REF', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --spawns melee > gpurun_out/bm.json 2> gpurun_out/bm.err || exit 4
python -c "import json; d=json.load(open('gpurun_out/bm.json')); print('MELEE', d['value']/1e6, 'M', d['roofline']['kernel_ms_mean']*1e3, 'us')"
LNW_PROF=1 timeout -k 10 300 python bench.py --steps 3 --warmup 5 --no-cpu-baseline --no-secondary --spawns melee > gpurun_out/pm.json 2> gpurun_out/pm.err || exit 5
grep "lnw prof" gpurun_out/pm.err | tail -2
grep "lnw prof" gpurun_out/pm.err | tail -1
