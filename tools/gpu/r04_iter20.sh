# round 4, iteration 20: the contact variant on the reference's recorded rollouts
# (tape mode, the rollout's fast path: row-less steps split by side, two-wave observe)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_rollout_golden.py > gpurun_out/t20.log 2>&1 || { tail -40 gpurun_out/t20.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/t20.log | tail -15
