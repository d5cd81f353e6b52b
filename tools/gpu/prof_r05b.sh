# round-5 rocprofv3 evidence, part 2: melee (contact variant), config 4, then
# config 5's kernel trace (tools/config5_profile.py: 8 rollouts x 40 steps)
set -o pipefail
bash tools/gpu/prof.sh r05_melee melee_e65536_los0_mv0 "--spawns melee" || exit 4
bash tools/gpu/prof.sh r05_config4 config4_e8192_los0_mv0 "--workload config4" || exit 5
export TMPDIR=/tmp
D=gpurun_out/r05_config5
rm -rf $D; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- python3 tools/config5_profile.py > $D/kt.log 2>&1 || exit 6
python3 tools/rocprof_summary.py r05_config5 --steps 320 --cmd "python3 tools/config5_profile.py (32 768 envs; 8 rollouts x 40 steps: 4 eager, 1 capture warm-up, 3 graph replays)" || exit 7
