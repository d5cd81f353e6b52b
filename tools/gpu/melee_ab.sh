# melee A/B: contact-variant kernel time with LNW_DEBUG_SKIP bits $1 (e.g. 131072 =
# per-lane bearing loop) against the default, interleaved, then the GPU tests
set -o pipefail
mkdir -p gpurun_out
B=${1:-131072}
for rep in 1 2; do
  for bits in 0 $B; do
    LNW_DEBUG_SKIP=$bits timeout -k 10 200 python bench.py --spawns melee --no-secondary --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/mab.json || exit 1
    python -c "import json;d=json.load(open('gpurun_out/mab.json'));print('bits $bits melee kernel ms', d['roofline']['kernel_ms_mean'])"
  done
done
