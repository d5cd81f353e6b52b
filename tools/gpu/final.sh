# round-end check: GPU test suite, smoke, and the default bench line with the
# CPU baseline and every secondary line (-> gpurun_out/bench_full.json)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tgpu.log 2>&1 || { tail -30 gpurun_out/tgpu.log; exit 1; }
tail -1 gpurun_out/tgpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench_full.json')); print(d['value']/1e9, 'G', d['roofline']); print({k: round(v.get('env_steps_per_sec', v.get('rays_per_sec', 0))/1e6, 1) for k, v in d['secondary'].items() if isinstance(v, dict)})"
