# round 6: lnw_policy_act with the tail loaded as float4 quads (actor_tq) against
# the per-value tail loads (actor_base): timing (tools/policy_probe.py, A/B/A/B)
# and determinism of the new build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/policy_probe.py tools/probe/actor_base.so tools/probe/actor_tq.so tools/probe/actor_base.so tools/probe/actor_tq.so tools/probe/actor_base.so tools/probe/actor_tq.so 2>&1 | grep "so {" || exit 1
POLICY_LIB=tools/probe/actor_tq.so timeout -k 10 300 python -u tools/policy_determinism.py 32768 40 packed,strided,critic > gpurun_out/det_tq.log 2>&1 || exit 2
grep "mismatching" gpurun_out/det_tq.log
