# round 4, iteration 6: grid timelines (headline, shards), shard PMC, melee epw
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/timeline.sh head "" || exit 1
bash tools/gpu/timeline.sh sh8192 "--global-envs 8192" || exit 2
bash tools/gpu/timeline.sh sh4096 "--global-envs 4096" || exit 3
for n in 8192 4096; do
  bash tools/gpu/pmc.sh f$n "FETCH_SIZE" "--global-envs $n" || exit 4
  bash tools/gpu/pmc.sh w$n "WRITE_SIZE" "--global-envs $n" || exit 5
done
echo "== melee epw"
for r in 1 2; do
  for e in 64 32 16; do
    LNW_EPW_RT=$e timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 100 --warmup 10 --spawns melee > gpurun_out/m.json 2>gpurun_out/m.err || { tail -5 gpurun_out/m.err; exit 6; }
    python -c "import json; d=json.load(open('gpurun_out/m.json')); print('melee epw $e', round(d['roofline']['kernel_ms_mean']*1e3, 1), 'us')"
  done
done
