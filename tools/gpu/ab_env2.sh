# A/B between LNW_DEBUG_SKIP values (arguments) at 65 536 and 8 192 envs, interleaved 3 times,
# after the GPU parity tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_rollout.py tests/test_gpu_facade.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tq.log 2>&1 || { tail -30 gpurun_out/tq.log; exit 1; }
tail -1 gpurun_out/tq.log
for r in 1 2 3; do
for B in "$@"; do
for GE in 65536 8192; do
LNW_DEBUG_SKIP=$B timeout -k 10 120 python bench.py --global-envs $GE --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 2
python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('skip', sys.argv[1], 'E', sys.argv[2], round(d['roofline']['kernel_ms_mean']*1e3,2), 'us')" $B $GE
done
done
done
