# round 6: the launch-time counter loads removed (they put 52 B/lane of scratch
# into the contact kernels and 28 B into the small-shard kernel) against the
# previous build; the GPU suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "--global-envs 8192" "--global-envs 4096" "" "--spawns melee" || exit $?
bash tools/gpu/tests.sh || exit $?
