# A/B of the default and melee bench lines over several builds given as arguments, interleaved
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for lib in "$@"; do
LNW_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
LNW_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-secondary --spawns melee > gpurun_out/abm.json 2> gpurun_out/abm.err || exit 2
python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); m=json.load(open('gpurun_out/abm.json')); print(sys.argv[1][-22:], 'REF', round(d['roofline']['kernel_ms_mean']*1e3,2), 'us  MELEE', round(m['roofline']['kernel_ms_mean']*1e3,1), 'us')" $lib
done
done
