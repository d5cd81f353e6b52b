# round 5: GPU suite + smoke, then the rollout / observe-split parity tests repeated 4 times
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/tests.sh || exit 1
for i in 1 2 3 4; do
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rollout_fullsize.py tests/test_gpu_rollout_golden.py tests/test_gpu_fullsize.py -k "contact or rollout" > gpurun_out/rep_$i.log 2>&1 || { tail -30 gpurun_out/rep_$i.log; exit 2; }
  tail -1 gpurun_out/rep_$i.log
done
