# round 5, first call: policy determinism map (all variants; the per-stage
# dump probe), then the new parity tests (shard direct mode, config-5 env side,
# medium snapshots, facade drawing)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/policy_determinism.py 32768 8 > gpurun_out/det_base.log 2>&1 || { tail -20 gpurun_out/det_base.log; exit 1; }
cat gpurun_out/det_base.log | grep -v "^lib"
POLICY_LIB=tools/probe/actor_dump.so PROBE_DUMP=1 timeout -k 10 240 python -u tools/policy_determinism.py 32768 8 packed,strided,strided_copy,packed_inplace > gpurun_out/det_dump.log 2>&1 || { tail -20 gpurun_out/det_dump.log; exit 2; }
cat gpurun_out/det_dump.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_state.py tests/test_gpu_facade.py tests/test_gpu_shard.py tests/test_gpu_rollout_fullsize.py > gpurun_out/t_new.log 2>&1 || { tail -40 gpurun_out/t_new.log; exit 3; }
tail -25 gpurun_out/t_new.log
bash tools/gpu/timeline.sh tl8192 "--global-envs 8192" || exit 4
bash tools/gpu/timeline.sh tl4096 "--global-envs 4096" || exit 5
