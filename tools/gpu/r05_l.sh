# round 5: strided policy input on; seq / rollout tests; bench with secondary lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_seq.py tests/test_gpu_rollout_golden.py tests/test_gpu_rollout.py tests/test_gpu_rollout_fullsize.py > gpurun_out/tests_l.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/tests_l.log | tail -30; exit 2; }
tail -3 gpurun_out/tests_l.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err || { tail -20 gpurun_out/bench_l.err; exit 3; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_l.json'))
print(d['value'], d['ms_per_step'])
for k,v in d['secondary'].items(): print(k, v.get('ms_per_step'), v.get('ms_per_rollout'), v.get('env_steps_per_sec'))"
