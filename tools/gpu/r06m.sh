# round 6: the quiet path compiled without phase S (timing probe,
# LNW_PROBE_QUIET_ONLY) against the production build, and its timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
bash tools/gpu/ab_lib.sh 2 $L tools/probe/liblnw_qonly.so "--global-envs 8192" "--global-envs 4096" "" || exit $?
LNW_LIB=$PWD/tools/probe/liblnw_qonly.so bash tools/gpu/timeline.sh qonly8192 "--global-envs 8192" 2>&1 | grep -E "quiet|grid:|qonly"
