# round 4, iteration 15: the contact variant's phase S split over both waves
# (LNW_SPLIT_S=1): contact-variant parity with it on, then melee A/B
set -o pipefail
export TMPDIR=/tmp
LNW_SPLIT_S=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_obs_options.py tests/test_gpu_state.py tests/test_gpu_fullsize.py \
  > gpurun_out/t15.log 2>&1 || { tail -30 gpurun_out/t15.log; exit 1; }
tail -3 gpurun_out/t15.log
bash tools/gpu/ab_env.sh LNW_SPLIT_S 3 "--spawns melee" || exit 2
