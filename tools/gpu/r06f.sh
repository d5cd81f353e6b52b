# round 6: policy probe 16, then config 4's fetch attribution (tools/gpu/c4_fetch.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/r06e.sh || exit 1
bash tools/gpu/c4_fetch.sh > gpurun_out/c4_fetch.txt 2>&1; rc=$?; cat gpurun_out/c4_fetch.txt; exit $rc
