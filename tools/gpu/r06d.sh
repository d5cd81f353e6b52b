# round 6, fourth call: policy probe 14 (inside the victim MLP: its fc1
# operands, its head outputs and per-row outputs against a rerun), then the
# rollout tests and config 5's kernel trace on the build with the critic's fc1
# loads all in flight
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
POLICY_LIB=tools/probe/actor_disturb14.so timeout -k 10 300 python -u tools/policy_determinism.py 32768 40 packed > gpurun_out/det_p14.log 2>&1
rc=$?; grep "^lib\|mismatching\|probe stage" gpurun_out/det_p14.log; fatal $rc && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout.py tests/test_gpu_rollout_golden.py tests/test_gpu_rollout_fullsize.py tests/test_gpu_obs_options.py > gpurun_out/ro_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ro_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/c5_trace.sh c5_post
