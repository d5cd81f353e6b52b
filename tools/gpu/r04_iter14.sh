# round 4, iteration 14: the group kernel's fire loop with the list entries side
# by side (fire_group_chunk): group parity, config 4 A/B against entry by entry
# (LNW_DEBUG_SKIP bit 15), section timers
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_group.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/t14.log 2>&1 || { tail -30 gpurun_out/t14.log; exit 1; }
tail -3 gpurun_out/t14.log
bash tools/gpu/ab_env.sh LNW_DEBUG_SKIP=32768 3 "--workload config4" || exit 2
bash tools/gpu/sections.sh c4 "--workload config4" || exit 3
