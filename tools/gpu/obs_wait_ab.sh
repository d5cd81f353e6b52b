# A/B: write_obs with the per-pass store wait (tools/probe/liblnw_ow.so) vs without (liblnw_base.so):
# config 5 rollout kernel times (observe / policy / step / post), then the rollout parity tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in liblnw_base.so liblnw_ow.so liblnw_base.so liblnw_ow.so; do
  LNW_LIB=$PWD/tools/probe/$lib timeout -k 10 300 python -u -c "
import sys, json; sys.argv = ['bench.py']; sys.path.insert(0, '.')
import bench
r = bench.mappo_rollout()
print('$lib', round(r['ms_per_rollout'], 3), 'ms per rollout', round(r['env_steps_per_sec'] / 1e6, 1), 'M')" 2>/dev/null || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout_fullsize.py tests/test_gpu_rollout_golden.py tests/test_gpu_rollout.py tests/test_gpu_obs_options.py > gpurun_out/ow_tests.log 2>&1 || { tail -20 gpurun_out/ow_tests.log; exit 2; }
tail -1 gpurun_out/ow_tests.log
