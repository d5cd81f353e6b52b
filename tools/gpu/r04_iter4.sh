# round 4, iteration 4: aligned 4-ship phase-S rows, MFMA critic, group-march A/B
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/tests.sh "rollout or policy or torch_impl or melee or units or facade or parity or headline or quiet" || exit 1
timeout -k 10 200 python tools/policy_probe.py littoral-naval-warfare-marl_amd/lnw/liblnw.so || exit 2
echo "== melee: line-aligned rows (0) vs row pieces (8192)"
bash tools/gpu/skip_ab.sh "--spawns melee" 0 8192 0 8192 || exit 3
for b in 0 8192; do
  LNW_LIB=$PWD/littoral-naval-warfare-marl_amd/lnw/liblnw_diag.so LNW_DEBUG_SKIP=$b bash tools/gpu/pmc.sh melee_w$b "WRITE_SIZE" "--spawns melee" || exit 4
done
echo "== config4 group march"
bash tools/gpu/ab_env.sh LNW_GROUP_MARCH 2 "--workload config4" || exit 5
echo "== headline / shards: unit-local barriers (0) vs workgroup barriers (LNW_UNIT_SYNC=1)"
bash tools/gpu/ab_env.sh LNW_UNIT_SYNC 3 "" "--global-envs 8192" || exit 6
