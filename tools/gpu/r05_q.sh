# round 5: contact-variant full-size parity repeated with the default (emission) path, then melee timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/contact_race.py 28 1 > gpurun_out/race_qj.log 2>&1 || { tail -20 gpurun_out/race_qj.log; exit 1; }
echo "default: clean runs: $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_qj.log) of 28"
grep -v amdgpu.ids gpurun_out/race_qj.log | grep -v " 0 hash" | grep -v "vs run 0: 0 " | head -8
for a in "--spawns melee" "--global-envs 4096 --spawns melee"; do
  timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 $a > gpurun_out/ab.json 2>/dev/null || exit 2
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$a', round(d['roofline']['kernel_ms_mean']*1e3, 2), 'us')"
done
