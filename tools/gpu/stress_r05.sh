# round-5 fixes under repetition: the split contact step's full-size rows (60 runs)
# and lnw_policy_act's outputs at 32 768 envs (150 repetitions per variant)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/contact_race.py 60 1 > gpurun_out/race_s.log 2>&1 || { tail -20 gpurun_out/race_s.log; exit 1; }
echo "contact split rows: clean runs $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_s.log) of 60"
timeout -k 10 900 python -u tools/policy_determinism.py 32768 150 critic,strided,packed > gpurun_out/det_s.log 2>&1 || { tail -20 gpurun_out/det_s.log; exit 2; }
grep "mismatching" gpurun_out/det_s.log
