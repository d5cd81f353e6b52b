# round 5: sequence kernels with laundered kernel arguments; seq tests + bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_seq.py tests/test_gpu_units.py > gpurun_out/tests_o.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/tests_o.log | tail -30; exit 2; }
tail -2 gpurun_out/tests_o.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench_o.json 2> gpurun_out/bench_o.err || { tail -20 gpurun_out/bench_o.err; exit 3; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_o.json'))
print(d['value'], d['ms_per_step'])
for k,v in d['secondary'].items(): print(k, v.get('ms_per_step'), v.get('kernel_ms'), v.get('ms_per_rollout'), v.get('env_steps_per_sec'))"
