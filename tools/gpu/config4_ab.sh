# config 4 (group kernel): the fix slopes four at a time (liblnw_s4.so) vs two (liblnw_base.so), then its parity tests
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/ab_lib.sh 2 tools/probe/liblnw_base.so tools/probe/liblnw_s4.so "--workload config4" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_fullsize.py -k "group or config4" > gpurun_out/c4_tests.log 2>&1 || { tail -20 gpurun_out/c4_tests.log; exit 2; }
tail -1 gpurun_out/c4_tests.log
