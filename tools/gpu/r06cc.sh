# the critic launch: 256-bound instantiation with the whole fc1 row prefetched (actor_new) vs HEAD (actor_prev), then determinism, rollout parity
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/policy_probe.py tools/probe/actor_prev.so tools/probe/actor_new.so tools/probe/actor_prev.so tools/probe/actor_new.so 2>&1 | grep -v amdgpu || exit 1
timeout -k 10 300 python -u tools/policy_determinism.py 32768 48 critic,strided,packed > gpurun_out/det_w.log 2>&1 || { tail -20 gpurun_out/det_w.log; exit 2; }
grep "mismatching" gpurun_out/det_w.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout_fullsize.py tests/test_gpu_rollout_golden.py tests/test_gpu_rollout.py tests/test_gpu_obs_options.py $(ls tests/test_gpu_*polic*.py tests/test_gpu_*actor*.py 2>/dev/null) > gpurun_out/w_tests.log 2>&1 || { tail -20 gpurun_out/w_tests.log; exit 3; }
tail -1 gpurun_out/w_tests.log
