# round-2 rocprofv3 evidence: headline, melee (contact variant), config 4,
# config 3's 8 192-env shard, and the march / A* mode (tools/gpu/prof.sh each)
set -o pipefail
bash tools/gpu/prof.sh r02_headline reference_e65536_los0_mv0 "" || exit 1
bash tools/gpu/prof.sh r02_melee melee_e65536_los0_mv0 "--spawns melee" || exit 2
bash tools/gpu/prof.sh r02_config4 config4_e8192_los0_mv0 "--workload config4" || exit 3
bash tools/gpu/prof.sh r02_shard8192 reference_e8192_los0_mv0 "--global-envs 8192" || exit 4
bash tools/gpu/prof.sh r02_march reference_e65536_los1_mv1 "--los-mode 1 --move-mode 1" || exit 5
