# round 6: final-build repetition evidence: split contact rows 60 runs, policy /
# critic 150 repetitions (tools/gpu/stress.sh), then the GPU suite a second time
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/stress.sh 60 150 || exit $?
bash tools/gpu/tests.sh || exit $?
