# quiet test timed twice (LNW_DEBUG_SKIP bit 24, diagnostics build): the second
# run of the same code shows what the first paid for instruction fetch
set -o pipefail
mkdir -p gpurun_out
for a in "--global-envs 8192" "--global-envs 4096" ""; do
  LNW_LIB=$PWD/littoral-naval-warfare-marl_amd/lnw/liblnw_diag.so LNW_PROF=1 LNW_DEBUG_SKIP=16777216 timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 2 --warmup 5 $a > gpurun_out/ic.json 2> gpurun_out/ic.err || { tail -5 gpurun_out/ic.err; exit 1; }
  echo "== $a"; grep "repeated quiet\|quiet workgroups" gpurun_out/ic.err | tail -2
done
export TMPDIR=/tmp
bash tools/gpu/pmc.sh ic8192 "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU" "--global-envs 8192" || exit 2
