# round 4, iteration 9: row-builder refactor vs previous build (melee, headline); config 5 line
set -o pipefail
export TMPDIR=/tmp
L=littoral-naval-warfare-marl_amd/lnw/liblnw.so
H=tools/probe/liblnw_head.so
bash tools/gpu/ab_lib.sh 2 $H $L "--spawns melee" "" "--global-envs 8192" || exit 1
timeout -k 10 300 python tools/config5_profile.py > gpurun_out/c5line.json 2> gpurun_out/c5line.err || { tail -5 gpurun_out/c5line.err; exit 2; }
cat gpurun_out/c5line.json
