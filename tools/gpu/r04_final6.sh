# round 4, final check after reverting the progress handoff (a contact full-size
# parity run failed once with it): GPU suite twice over the contact tests, then the
# round-end check
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fullsize.py \
  tests/test_gpu_obs_options.py > gpurun_out/t25.log 2>&1 || { tail -30 gpurun_out/t25.log; exit 1; }
tail -1 gpurun_out/t25.log
bash tools/gpu/final.sh || exit 2
