# round 4, third final pass (observe on two waves, the rollout step split by side):
# headline profile (traffic.json keyed to the current sources), config 5's kernel
# trace, then the round-end check
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/prof.sh r04_headline reference_e65536_los0_mv0 "" || exit 1
D=gpurun_out/r04_config5
rm -rf $D; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- python3 tools/config5_profile.py > $D/kt.log 2>&1 || exit 2
bash tools/gpu/final.sh || exit 3
