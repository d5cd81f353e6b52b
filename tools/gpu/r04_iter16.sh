# round 4, iteration 16: config 4 — fixes two divisions in flight (lnw_c4_fix.so)
# and target lists staged in LDS during phase S (current build): group parity,
# then interleaved A/B of base / fix / current
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_group.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_state.py > gpurun_out/t16.log 2>&1 || { tail -30 gpurun_out/t16.log; exit 1; }
tail -2 gpurun_out/t16.log
for r in 1 2 3; do
  for lib in tools/probe/lnw_c4_base.so tools/probe/lnw_c4_fix.so littoral-naval-warfare-marl_amd/lnw/liblnw.so; do
    LNW_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 --workload config4 \
      > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 2; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('r$r', '$(basename $lib)', round(d['roofline']['kernel_ms_mean']*1e3, 2), 'us')"
  done
done
