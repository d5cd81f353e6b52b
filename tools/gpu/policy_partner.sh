# lnw_policy_act determinism under each partner-wave probe (tools/build_probes.sh:
# LNW_PROBE_DISTURB modes), then the bench line with its secondary lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/det_m.log
for d in 1 2 3 4 5 6 7 8 9 10 11 12; do
  POLICY_LIB=tools/probe/actor_disturb$d.so timeout -k 10 200 python -u tools/policy_determinism.py 32768 40 packed,strided >> gpurun_out/det_m.log 2>&1 || { tail -20 gpurun_out/det_m.log; exit 1; }
done
grep "^lib\|mismatching" gpurun_out/det_m.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench_m.json 2> gpurun_out/bench_m.err || { tail -20 gpurun_out/bench_m.err; exit 3; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_m.json'))
print(d['value'], d['ms_per_step'])
for k,v in d['secondary'].items(): print(k, v.get('ms_per_step'), v.get('kernel_ms'), v.get('ms_per_rollout'), v.get('env_steps_per_sec'))"
