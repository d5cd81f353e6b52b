# round 5: split contact rows with the per-pass store wait (production build): parity repeated, then the GPU suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
RACE_REF_NOSPLIT=1 timeout -k 10 900 python -u tools/contact_race.py 30 1 > gpurun_out/race_v.log 2>&1 || { tail -20 gpurun_out/race_v.log; exit 1; }
echo "clean runs: $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_v.log) of 30"
grep -v amdgpu.ids gpurun_out/race_v.log | grep -v " 0 hash" | grep -v "vs run 0: 0 " | head -8
bash tools/gpu/tests.sh
