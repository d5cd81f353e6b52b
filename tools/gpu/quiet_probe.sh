# headline kernel time vs episode horizon (fewer non-quiet workgroups at shorter horizons)
set -o pipefail
for H in 40 20 10; do
  timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 --episode-steps $H > gpurun_out/qp_$H.json 2>/dev/null || exit 1
  LNW_PROF=1 timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 40 --warmup 5 --episode-steps $H 2>&1 >/dev/null | grep "quiet workgroups" | awk '{print $4}' | sort -n | uniq -c | tr '\n' ' ' > gpurun_out/qp_$H.txt
  python -c "import json;d=json.load(open('gpurun_out/qp_$H.json'));print('horizon',$H,round(d['roofline']['kernel_ms_mean']*1e3,2),'us; quiet WG counts per launch (count x value):',open('gpurun_out/qp_$H.txt').read())"
done
