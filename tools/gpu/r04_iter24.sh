# round 4, iteration 24: the split contact kernel with a per-ship progress handoff instead of
# the first barrier: contact parity, then melee / config 5
# A/B against the previous build (tools/probe/lnw_base.so)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_obs_options.py tests/test_gpu_parity.py tests/test_gpu_state.py tests/test_gpu_fullsize.py \
  tests/test_gpu_rollout.py tests/test_gpu_rollout_golden.py > gpurun_out/t24.log 2>&1 || { tail -40 gpurun_out/t24.log; exit 1; }
tail -2 gpurun_out/t24.log
for r in 1 2; do
  for lib in tools/probe/lnw_base.so littoral-naval-warfare-marl_amd/lnw/liblnw.so; do
    LNW_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 100 --warmup 10 --spawns melee \
      > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 3; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('r$r', '$(basename $lib)', 'melee', round(d['roofline']['kernel_ms_mean']*1e3, 2), 'us')"
  done
done
LNW_LIB=$PWD/littoral-naval-warfare-marl_amd/lnw/liblnw.so timeout -k 10 300 python tools/config5_profile.py > gpurun_out/c5ab.json 2> gpurun_out/c5ab.err || { tail -5 gpurun_out/c5ab.err; exit 2; }
python -c "import json; d=json.load(open('gpurun_out/c5ab.json')); print('config5', round(d['env_steps_per_sec']/1e6, 1), 'M')"
