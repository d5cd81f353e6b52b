# round 4, fourth final pass (contact phase S split by side): profiles for the
# headline (traffic.json keyed to the current sources), melee and config 5, then
# the round-end check
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/prof.sh r04_headline reference_e65536_los0_mv0 "" || exit 1
bash tools/gpu/prof.sh r04_melee melee_e65536_los0_mv0 "--spawns melee" || exit 2
D=gpurun_out/r04_config5
rm -rf $D; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- python3 tools/config5_profile.py > $D/kt.log 2>&1 || exit 3
bash tools/gpu/final.sh || exit 4
