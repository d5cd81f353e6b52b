# round 6: the small shards' row stores without write-through (LNW_NO_STORE_WT:
# plain stores), interleaved A/B of the knob
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/ab_env.sh LNW_NO_STORE_WT 3 "--global-envs 8192" "--global-envs 4096" "" || exit $?
