# round 6: config 4's rows with batched window loads: A/B against the previous
# build (tools/probe/liblnw_prev.so), then the group-kernel parity tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so littoral-naval-warfare-marl_amd/lnw/liblnw.so "--workload config4" || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_fullsize.py tests/test_gpu_crash_modes.py tests/test_gpu_state.py > gpurun_out/grp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/grp_tests.log; exit $rc
