# round 4, second final pass (group kernel fire loop): profiles for the headline
# (traffic.json keyed to the current sources) and config 4, then the round-end check
set -o pipefail
bash tools/gpu/prof.sh r04_headline reference_e65536_los0_mv0 "" || exit 1
bash tools/gpu/prof.sh r04_config4 config4_e8192_los0_mv0 "--workload config4" || exit 2
bash tools/gpu/final.sh || exit 3
