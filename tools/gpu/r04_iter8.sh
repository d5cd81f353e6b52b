# round 4, iteration 8: red rewards on wave 1 (small quiet workgroups); group kernel for 4v4 (A/B)
set -o pipefail
export TMPDIR=/tmp
L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
H=tools/probe/liblnw_head.so
bash tools/gpu/tests.sh "quiet or parity or units or golden or state or shard or config2 or small" || exit 1
bash tools/gpu/ab_lib.sh 3 $H $L "--global-envs 8192" "--global-envs 4096" || exit 3
echo "== melee: group kernel (1) vs contact variant (0)"
bash tools/gpu/ab_env.sh LNW_FORCE_GROUP 1 "--spawns melee" || exit 4
LNW_FORCE_GROUP=1 bash tools/gpu/c5_trace.sh c5_grp || exit 5
