# Repetition checks of the two kernels whose faults were intermittent: the split
# contact step's full-size rows (tools/contact_race.py, N runs) and
# lnw_policy_act / the critic at 32 768 envs (tools/policy_determinism.py):
#   bash tools/gpu/stress.sh [N=60] [REPS=150]
set -o pipefail
N=${1:-60}; REPS=${2:-150}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/contact_race.py $N 1 > gpurun_out/race_stress.log 2>&1 || { tail -20 gpurun_out/race_stress.log; exit 1; }
echo "contact split rows: clean runs $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_stress.log) of $N"
timeout -k 10 900 python -u tools/policy_determinism.py 32768 $REPS critic,strided,packed > gpurun_out/det_stress.log 2>&1 || { tail -20 gpurun_out/det_stress.log; exit 2; }
grep "mismatching" gpurun_out/det_stress.log
