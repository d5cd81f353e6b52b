# round 6: small quiet workgroups without the phase-Q barrier (wave 1 commits
# every move itself, wave 0 takes the final cells from the phase-M columns)
# against the previous build, the whole GPU suite, the 8 192-env timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 8192" "--global-envs 4096" "--global-envs 16384" || exit $?
bash tools/gpu/tests.sh || exit $?
bash tools/gpu/timeline.sh sh8192n "--global-envs 8192" 2>&1 | grep -E "quiet|grid:|sh8192n"
