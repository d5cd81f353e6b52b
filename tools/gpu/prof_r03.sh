# round-3 rocprofv3 evidence (tools/gpu/prof.sh each): headline (units kernel),
# config 3's 8 192-env shard, config 2, melee (contact variant), config 4, then
# config 5's kernel trace (tools/config5_profile.py: 8 rollouts x 40 steps)
set -o pipefail
bash tools/gpu/prof.sh r03_headline reference_e65536_los0_mv0 "" || exit 1
bash tools/gpu/prof.sh r03_shard8192 reference_e8192_los0_mv0 "--global-envs 8192" || exit 2
bash tools/gpu/prof.sh r03_config2 reference_e4096_los0_mv0 "--global-envs 4096" || exit 3
bash tools/gpu/prof.sh r03_melee melee_e65536_los0_mv0 "--spawns melee" || exit 4
bash tools/gpu/prof.sh r03_config4 config4_e8192_los0_mv0 "--workload config4" || exit 5
export TMPDIR=/tmp
D=gpurun_out/r03_config5
rm -rf $D; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- python3 tools/config5_profile.py > $D/kt.log 2>&1 || exit 6
python3 tools/rocprof_summary.py r03_config5 --steps 320 --cmd "python3 tools/config5_profile.py (32 768 envs; 8 rollouts x 40 steps: 4 eager, 1 capture warm-up, 3 graph replays)" || exit 7
