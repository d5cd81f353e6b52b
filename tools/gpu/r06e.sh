# round 6: policy probes 15 (layers per row tile vs a rerun) and 16 (fc1 split terms, pre-activation)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
POLICY_LIB=tools/probe/actor_disturb16.so timeout -k 10 300 python -u tools/policy_determinism.py 32768 20 packed > gpurun_out/det_p16.log 2>&1
rc=$?; grep "^lib\|mismatching\|probe stage" gpurun_out/det_p16.log; exit $rc
