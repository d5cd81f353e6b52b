# the GPU suite twice in a row (flakiness check), then smoke
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:randomly > gpurun_out/suite_$i.log 2>&1
  rc=$?
  tail -1 gpurun_out/suite_$i.log
  grep -E "^FAILED|^ERROR" gpurun_out/suite_$i.log | head -5
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
