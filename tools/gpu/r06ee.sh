# round 6: the quiet branch marked likely (block placement) against the previous
# build: interleaved A/B at the headline and the shard sizes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "" "--global-envs 8192" "--global-envs 4096" || exit $?
