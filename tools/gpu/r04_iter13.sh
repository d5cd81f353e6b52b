# round 4, iteration 13: two passes in flight per wave in the quiet units' stream
# (LNW_EMIT_DEPTH=2): parity of the units kernel with it on, then interleaved A/B
set -o pipefail
export TMPDIR=/tmp
LNW_EMIT_DEPTH=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_units.py tests/test_gpu_obs_options.py > gpurun_out/t13.log 2>&1 || { tail -30 gpurun_out/t13.log; exit 1; }
tail -3 gpurun_out/t13.log
bash tools/gpu/ab_env.sh LNW_EMIT_DEPTH=2 4 "" "--global-envs 8192" || exit 2
