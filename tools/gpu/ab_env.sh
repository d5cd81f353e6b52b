# A/B of the headline kernel between LNW_DEBUG_SKIP values (argument list), interleaved 3 times
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
for B in "$@"; do
LNW_DEBUG_SKIP=$B timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 2
python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('skip', sys.argv[1], 'REF', round(d['roofline']['kernel_ms_mean']*1e3,2), 'us')" $B
done
done
