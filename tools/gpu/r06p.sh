# round 6: small quiet workgroups' env / draw counters loaded at launch, A/B of
# the knob (LNW_DEBUG_SKIP bit 29 = loaded in phase Q) at the shard sizes of
# N = 16 / 8 / 4 GPUs, then the quiet-path tests and the 4 096-env timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/ab_env.sh LNW_DEBUG_SKIP=536870912 3 "--global-envs 4096" "--global-envs 8192" "--global-envs 16384" || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_state.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/timeline.sh sh4096n "--global-envs 4096" 2>&1 | grep -E "quiet|grid:|sh4096n"
LNW_DEBUG_SKIP=536870912 bash tools/gpu/timeline.sh sh4096q "--global-envs 4096" 2>&1 | grep -E "quiet|grid:|sh4096q"
