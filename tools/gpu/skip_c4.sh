# config 4 kernel time with diagnostics sections skipped (LNW_DEBUG_SKIP bits)
set -o pipefail
for B in ${BITS:-0 1 128 256 384 2}; do
  LNW_DEBUG_SKIP=$B timeout -k 10 120 python bench.py --workload config4 --no-secondary --no-cpu-baseline --steps 60 --warmup 10 > gpurun_out/sk_$B.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sk_$B.json'));print('skip',$B,round(d['roofline']['kernel_ms_mean']*1e3,1),'us')"
done
