# round 6, second call: the phase-O race on the shipped code minus its store
# wait (tools/probe/liblnw_nowait.so, -DLNW_PROBE_NO_OBS_WAIT) with every wrong
# block dumped; the GPU suite; config 5's per-launch PMC; the default bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
RACE_REF_NOSPLIT=1 RACE_DUMP=gpurun_out/race_dump_nowait.npz LNW_LIB=$PWD/tools/probe/liblnw_nowait.so \
  timeout -k 10 600 python -u tools/contact_race.py 60 1 > gpurun_out/race_nowait.log 2>&1
rc=$?; echo "no-wait race: clean runs $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_nowait.log) of 60"
grep "dumped" gpurun_out/race_nowait.log; fatal $rc && exit $rc
bash tools/gpu/tests.sh; rc=$?; fatal $rc && exit $rc
bash tools/gpu/c5_pmc.sh r06_config5; rc=$?; fatal $rc && exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r06b.json 2> gpurun_out/bench_r06b.err
rc=$?; tail -c 600 gpurun_out/bench_r06b.json; exit $rc
