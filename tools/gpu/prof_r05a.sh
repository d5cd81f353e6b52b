# round-5 rocprofv3 evidence, part 1 (tools/gpu/prof.sh each): headline (units
# kernel), config 3's 8 192-env shard, config 2
set -o pipefail
bash tools/gpu/prof.sh r05_headline reference_e65536_los0_mv0 "" || exit 1
bash tools/gpu/prof.sh r05_shard8192 reference_e8192_los0_mv0 "--global-envs 8192" || exit 2
bash tools/gpu/prof.sh r05_config2 reference_e4096_los0_mv0 "--global-envs 4096" || exit 3
