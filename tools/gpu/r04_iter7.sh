# round 4, iteration 7: quiet-tail fast path and the policy's obs-copy placement vs HEAD
set -o pipefail
export TMPDIR=/tmp
L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
H=tools/probe/liblnw_head.so
bash tools/gpu/tests.sh "quiet or parity or units or golden or state or shard or rollout" || exit 1
timeout -k 10 200 python tools/policy_probe.py $H $L $H $L || exit 2
bash tools/gpu/ab_lib.sh 3 $H $L "" "--global-envs 8192" "--global-envs 4096" || exit 3
