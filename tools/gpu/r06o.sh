# round 6: env and draw counters loaded at launch in small quiet workgroups
# against the previous build: interleaved A/B, the quiet-path tests, timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 8192" "--global-envs 4096" "" || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_state.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tk.log 2>&1; rc=$?; tail -3 gpurun_out/tk.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/timeline.sh sh8192n "--global-envs 8192" 2>&1 | grep -E "quiet|grid:|sh8192n"
