# A/B of the headline kernel over builds given as arguments, interleaved 3 times,
# after the quiet-path and parity GPU tests on the in-tree build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tq.log 2>&1 || { tail -30 gpurun_out/tq.log; exit 1; }
tail -1 gpurun_out/tq.log
for r in 1 2 3; do
for lib in "$@"; do
LNW_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 2
python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[1][-16:], 'REF', round(d['roofline']['kernel_ms_mean']*1e3,2), 'us')" $lib
done
done
