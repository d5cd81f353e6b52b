# round 5: what the partner wave of a SIMD does while a wave runs its MLP
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/det_m.log
for d in 6 7 8 9; do
  POLICY_LIB=tools/probe/actor_disturb$d.so timeout -k 10 200 python -u tools/policy_determinism.py 32768 40 packed,strided >> gpurun_out/det_m.log 2>&1 || { tail -20 gpurun_out/det_m.log; exit 1; }
done
grep "^lib\|mismatching" gpurun_out/det_m.log
