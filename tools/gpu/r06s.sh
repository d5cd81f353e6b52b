# round 6: what phase M's double sincos costs (timing probe with an f32
# __sincosf in its place, results change) at the headline and the shard sizes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
bash tools/gpu/ab_lib.sh 3 $L tools/probe/liblnw_fastsc.so "" "--global-envs 8192" "--global-envs 4096" || exit $?
