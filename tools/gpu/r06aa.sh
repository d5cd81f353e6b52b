# round 6 final evidence, part A: the GPU suite + smoke(), the stress runs
# (split contact rows 30x, policy / critic determinism), the rocprofv3 evidence
# of the headline, the 8 192-env shard and config 2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/tests.sh || exit $?
bash tools/gpu/stress.sh 30 48 || exit $?
bash tools/gpu/prof_all.sh r06 1 || exit $?
