# round 6: crash-mode parity + the GPU suite, then the phase-O race without its
# per-pass store wait (diagnostics build, LNW_DEBUG_SKIP bit 25) with every wrong
# block dumped for the offline source attribution (tools/race_chunks.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_crash_modes.py -x -v --timeout 300 --timeout-method thread > gpurun_out/crash.log 2>&1
rc=$?; tail -5 gpurun_out/crash.log; fatal $rc && exit $rc
bash tools/gpu/tests.sh; rc=$?; fatal $rc && exit $rc
RACE_REF_NOSPLIT=1 RACE_SKIP_BITS=33554432 RACE_DUMP=gpurun_out/race_dump.npz \
  LNW_LIB=$PWD/littoral-naval-warfare-marl_amd/lnw/liblnw_diag.so \
  timeout -k 10 600 python -u tools/contact_race.py 10 1 > gpurun_out/race_r06.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/race_r06.log | grep "^run\|dumped" | head -12
exit $rc
