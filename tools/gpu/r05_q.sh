# round 5: contact-variant full-size parity repeated: wave 1 resident through phase O (diagnostics build) vs default
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LNW_LIB=tools/probe/liblnw_stay.so timeout -k 10 900 python -u tools/contact_race.py 28 1 > gpurun_out/race_qh.log 2>&1 || { tail -20 gpurun_out/race_qh.log; exit 1; }
echo "stay: clean runs: $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_qh.log) of 28"
grep -v amdgpu.ids gpurun_out/race_qh.log | grep -v " 0 hash" | grep -v "vs run 0: 0 " | head -8
timeout -k 10 900 python -u tools/contact_race.py 28 1 > gpurun_out/race_qi.log 2>&1 || { tail -20 gpurun_out/race_qi.log; exit 1; }
echo "default (vmcnt wait): clean runs: $(grep -c ' 0 hash, 0 reward, 0 done' gpurun_out/race_qi.log) of 28"
grep -v amdgpu.ids gpurun_out/race_qi.log | grep -v " 0 hash" | grep -v "vs run 0: 0 " | head -8
