# A round's rocprofv3 evidence (tools/gpu/prof.sh per workload, then config 5 by
# tools/gpu/c5_pmc.sh):  bash tools/gpu/prof_all.sh r06 [part]
#   part 1: headline (units kernel), config 3's 8 192- and 16 384-env shards, config 2
#   part 2: melee (contact variant), config 4, config 5        (default: both)
set -o pipefail
R=${1:?round tag, e.g. r06}; PART=${2:-all}
if [ "$PART" = all ] || [ "$PART" = 1 ]; then
  bash tools/gpu/prof.sh ${R}_headline reference_e65536_los0_mv0 "" || exit 1
  bash tools/gpu/prof.sh ${R}_shard8192 reference_e8192_los0_mv0 "--global-envs 8192" || exit 2
  bash tools/gpu/prof.sh ${R}_config2 reference_e4096_los0_mv0 "--global-envs 4096" || exit 3
  bash tools/gpu/prof.sh ${R}_shard16384 reference_e16384_los0_mv0 "--global-envs 16384" || exit 7
fi
if [ "$PART" = all ] || [ "$PART" = 2 ]; then
  bash tools/gpu/prof.sh ${R}_melee melee_e65536_los0_mv0 "--spawns melee" || exit 4
  bash tools/gpu/prof.sh ${R}_config4 config4_e8192_los0_mv0 "--workload config4" || exit 5
  bash tools/gpu/c5_pmc.sh ${R}_config5 || exit 6
fi
