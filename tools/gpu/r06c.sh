# round 6, third call: the phase-O fault's dependence on write-through stores
# (the no-wait probe with LNW_NO_STORE_WT: non-temporal global stores instead of
# buffer_store ... sc1), the shipped build repeated, and the policy tile
# read-back probe (13) beside the fault's reproduction (probe 10)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
LNW_NO_STORE_WT=1 RACE_REF_NOSPLIT=1 RACE_DUMP=gpurun_out/race_dump_nowait_nt.npz LNW_LIB=$PWD/tools/probe/liblnw_nowait.so \
  timeout -k 10 600 python -u tools/contact_race.py 60 1 > gpurun_out/race_nowait_nt.log 2>&1
rc=$?; echo "no-wait, non-temporal stores: clean runs $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_nowait_nt.log) of 60"; fatal $rc && exit $rc
timeout -k 10 600 python -u tools/contact_race.py 60 1 > gpurun_out/race_prod.log 2>&1
rc=$?; echo "shipped (wait, write-through): clean runs $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_prod.log) of 60"; fatal $rc && exit $rc
: > gpurun_out/det_p13.log
for d in 10 13; do
  POLICY_LIB=tools/probe/actor_disturb$d.so timeout -k 10 300 python -u tools/policy_determinism.py 32768 40 packed,strided >> gpurun_out/det_p13.log 2>&1
  rc=$?; fatal $rc && exit $rc
done
grep "^lib\|mismatching\|probe stage" gpurun_out/det_p13.log
