# round 5: serialized per-SIMD MLP phases in liblnw.so; determinism + policy/rollout/seq tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/policy_determinism.py 32768 64 critic,strided_nolive,packed_inplace,strided,packed > gpurun_out/det_k.log 2>&1 || { tail -20 gpurun_out/det_k.log; exit 1; }
grep "mismatching" gpurun_out/det_k.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_obs_options.py tests/test_gpu_seq.py tests/test_gpu_rollout_golden.py tests/test_gpu_rollout.py > gpurun_out/tests_k.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/tests_k.log | tail -30; exit 2; }
tail -3 gpurun_out/tests_k.log
