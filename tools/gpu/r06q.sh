# round 6 evidence, part A: the GPU suite + smoke(), then the rocprofv3 evidence
# of the headline, the 8 192-env shard and config 2 (prof_all.sh part 1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/tests.sh || exit $?
bash tools/gpu/prof_all.sh r06 1 || exit $?
