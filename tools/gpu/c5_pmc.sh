# rocprofv3 evidence for config 5 (tools/config5_profile.py: 32 768-env MAPPO
# rollouts): kernel trace + stats, then FETCH_SIZE, WRITE_SIZE and an SQ group in
# passes of their own, summarised per launch family into profiles/$TAG_rocprof.md
#   bash tools/gpu/c5_pmc.sh r06_config5
set -o pipefail
TAG=${1:-r06_config5}
export TMPDIR=/tmp
mkdir -p gpurun_out
D=gpurun_out/$TAG
rm -rf $D; mkdir -p $D
C="tools/config5_profile.py"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- python3 $C > $D/kt.log 2>&1 || { tail -20 $D/kt.log; exit 2; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/fetch -o fetch --output-format csv -- python3 $C > $D/fetch.log 2>&1 || { tail -5 $D/fetch.log; exit 3; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/write -o write --output-format csv -- python3 $C > $D/write.log 2>&1 || { tail -5 $D/write.log; exit 4; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d $D/sq -o sq --output-format csv -- python3 $C > $D/sq.log 2>&1 || { tail -5 $D/sq.log; exit 5; }
python3 tools/rocprof_summary.py $TAG --config5 --envs 32768 --cmd "python3 $C (32 768 envs; 8 rollouts x 40 steps: 4 eager, 1 capture warm-up, 3 graph replays)" || exit 7
