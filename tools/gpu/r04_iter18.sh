# round 4, iteration 18: the contact variant's observe kernel on four waves of 64 envs (half a
# side's calls each, past the earlier ships' draws): observe / rollout parity,
# then config 5 A/B (tools/probe/lnw_obs2.so = the two-wave build) and the observe
# kernel time under a kernel trace
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_obs_options.py tests/test_gpu_parity.py tests/test_gpu_state.py tests/test_gpu_rollout.py \
  tests/test_gpu_rollout_golden.py tests/test_gpu_fullsize.py > gpurun_out/t18.log 2>&1 || { tail -30 gpurun_out/t18.log; exit 1; }
tail -2 gpurun_out/t18.log
for r in 1 2; do
  for lib in tools/probe/lnw_obs2.so littoral-naval-warfare-marl_amd/lnw/liblnw.so; do
    LNW_LIB=$PWD/$lib timeout -k 10 300 python tools/config5_profile.py > gpurun_out/c5ab.json 2> gpurun_out/c5ab.err || { tail -5 gpurun_out/c5ab.err; exit 2; }
    python -c "import json; d=json.load(open('gpurun_out/c5ab.json')); print('r$r', '$(basename $lib)', round(d['env_steps_per_sec']/1e6, 1), 'M')"
  done
done
D=gpurun_out/c5_obs4; rm -rf $D; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- python3 tools/config5_profile.py > $D/kt.log 2>&1 || exit 3
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/c5_obs4/kt/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
