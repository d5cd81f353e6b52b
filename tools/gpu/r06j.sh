# round 6: LNW_PROF timelines of the small shards (production build)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/timeline.sh sh8192 "--global-envs 8192" || exit $?
bash tools/gpu/timeline.sh sh4096 "--global-envs 4096" || exit $?
