# round 6: the policy fault against the split-before-MFMA fence: probe 10's
# schedule (the partner's head beside each MLP) and the overlapped schedule
# (each wave's MLP right after its own head) with and without the fence, then
# the timing of base / fence / overlap+fence (tools/policy_probe.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/det_fence.log
for v in disturb10 disturb10_fence overlap overlap_fence fence; do
  POLICY_LIB=tools/probe/actor_$v.so timeout -k 10 300 python -u tools/policy_determinism.py 32768 40 packed,strided >> gpurun_out/det_fence.log 2>&1 || exit 1
done
grep "^lib\|mismatching" gpurun_out/det_fence.log
timeout -k 10 300 python -u tools/policy_probe.py tools/probe/actor_base.so tools/probe/actor_fence.so tools/probe/actor_overlap_fence.so tools/probe/actor_base.so tools/probe/actor_fence.so tools/probe/actor_overlap_fence.so 2>&1 | grep "so {" 
