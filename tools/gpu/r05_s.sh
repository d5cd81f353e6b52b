# round 5: the early quiet test -- parity tests, then interleaved A/B against the previous build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_units.py tests/test_gpu_fullsize.py tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_seq.py > gpurun_out/tests_s.log 2>&1 || { tail -30 gpurun_out/tests_s.log; exit 1; }
tail -1 gpurun_out/tests_s.log
bash tools/gpu/ab_lib.sh 3 tools/probe/liblnw_base.so tools/probe/liblnw_eq.so "--global-envs 8192" "--global-envs 4096" "" || exit 2
