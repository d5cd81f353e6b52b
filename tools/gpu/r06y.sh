# round 6: the launch-time counter loads kept in the non-contact kernels only
# (the contact variants scratch-free again) against the previous build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 8192" "--spawns melee" "" || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_state.py tests/test_gpu_rollout.py tests/test_gpu_rollout_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; exit $rc
