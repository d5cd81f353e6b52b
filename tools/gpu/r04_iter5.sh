set -o pipefail
timeout -k 10 200 python tools/policy_probe.py littoral-naval-warfare-marl_amd/lnw/liblnw.so tools/probe/actor_base.so tools/probe/actor_NOCONV.so tools/probe/actor_NOMLP.so || exit 1
export TMPDIR=/tmp
echo "== melee: line-aligned rows (0) vs row pieces (8192)"
bash tools/gpu/skip_ab.sh "--spawns melee" 0 8192 0 8192 || exit 3
for b in 0 8192; do
  LNW_LIB=$PWD/littoral-naval-warfare-marl_amd/lnw/liblnw_diag.so LNW_DEBUG_SKIP=$b bash tools/gpu/pmc.sh melee_w$b "WRITE_SIZE" "--spawns melee" || exit 4
done
echo "== config4 group march"
bash tools/gpu/ab_env.sh LNW_GROUP_MARCH 2 "--workload config4" || exit 5
echo "== config 5 kernel trace: default epw, then 64"
bash tools/gpu/c5_trace.sh c5_def || exit 7
LNW_EPW_RT=64 bash tools/gpu/c5_trace.sh c5_e64 || exit 8
