# One build-measure iteration: the GPU test suite, then kernel times of the
# given bench workloads (production build):  bash tools/gpu/iter.sh "ARGS" ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tgpu.log 2>&1 || { tail -40 gpurun_out/tgpu.log; exit 1; }
tail -2 gpurun_out/tgpu.log
for args in "$@"; do
  timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 100 --warmup 10 $args > gpurun_out/it.json 2>/dev/null || exit 2
  python -c "import json; d=json.load(open('gpurun_out/it.json')); print('$args', round(d['value']/1e6, 2), 'M env-steps/s', round(d['roofline']['kernel_ms_mean']*1e3, 1), 'us')"
done
