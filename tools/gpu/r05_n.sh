# round 5: partner wave redoes its head while a wave runs its MLP
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/det_n.log
for d in 12; do POLICY_LIB=tools/probe/actor_disturb$d.so timeout -k 10 200 python -u tools/policy_determinism.py 32768 20 packed,strided >> gpurun_out/det_n.log 2>&1 || { tail -20 gpurun_out/det_n.log; exit 1; }; done
grep "^lib\|mismatching\|probe" gpurun_out/det_n.log
