# round 4, iteration 12: determinism diagnosis, rollout default path, full GPU suite, config 5
set -o pipefail
export TMPDIR=/tmp
POLICY_LIB=$PWD/tools/probe/actor_base.so timeout -k 10 200 python tools/policy_determinism.py 32768 8 strided,packed || exit 1
POLICY_LIB=$PWD/tools/probe/actor_wz.so timeout -k 10 200 python tools/policy_determinism.py 32768 8 strided,packed || exit 2
timeout -k 10 300 python tools/rollout_determinism.py 32768 40 1 direct,direct,direct,callback || exit 3
bash tools/gpu/tests.sh || exit 4
bash tools/gpu/c5_trace.sh c5_r04 || exit 5
timeout -k 10 300 python tools/config5_profile.py > gpurun_out/c5line.json 2> gpurun_out/c5line.err || { tail -5 gpurun_out/c5line.err; exit 6; }
cat gpurun_out/c5line.json
