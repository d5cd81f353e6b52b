# round 4, iteration 10: rollout without redundant observation copies / rows
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/tests.sh "obs_options or rollout or policy or torch_impl" || exit 1
bash tools/gpu/c5_trace.sh c5_direct || exit 2
timeout -k 10 300 python tools/config5_profile.py > gpurun_out/c5line.json 2> gpurun_out/c5line.err || { tail -5 gpurun_out/c5line.err; exit 3; }
cat gpurun_out/c5line.json
echo "== shard epw"
for n in 8192 4096; do for e in 8 16 32; do
  LNW_EPW_RT=$e timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 --global-envs $n > gpurun_out/e.json 2>gpurun_out/e.err || { tail -5 gpurun_out/e.err; exit 4; }
  python -c "import json; d=json.load(open('gpurun_out/e.json')); print('envs $n epw $e', round(d['roofline']['kernel_ms_mean']*1e3, 2), 'us')"
done; done
