# round 6: float32 move rows: target cell from float polynomials when its rounding
# is certain (move_cell_f32_fast; the double sincos otherwise) against the
# previous build, then the whole GPU suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_prev.so $L "" "--global-envs 8192" "--global-envs 4096" "--spawns melee" || exit $?
bash tools/gpu/tests.sh || exit $?
