# rocprofv3 evidence for one bench workload: kernel trace + stats, then one run
# per PMC group (FETCH_SIZE and WRITE_SIZE in passes of their own, SQ groups
# within the per-block limits), then the summary into profiles/.
#   bash tools/gpu/prof.sh TAG KEY "BENCH ARGS"
# e.g. bash tools/gpu/prof.sh r02_headline reference_e65536_los0_mv0 ""
set -o pipefail
TAG=$1; KEY=$2; ARGS=$3
mkdir -p gpurun_out
export TMPDIR=/tmp
D=gpurun_out/$TAG
rm -rf $D; mkdir -p $D
B="bench.py --no-secondary --no-cpu-baseline $ARGS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- python3 $B --steps 200 --warmup 20 > $D/kt.log 2>&1 || exit 2
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/fetch -o fetch --output-format csv -- python3 $B --steps 30 --warmup 5 > $D/fetch.log 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/write -o write --output-format csv -- python3 $B --steps 30 --warmup 5 > $D/write.log 2>&1 || exit 4
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $D/sq -o sq --output-format csv -- python3 $B --steps 30 --warmup 5 > $D/sq.log 2>&1 || exit 5
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM --kernel-trace -d $D/sq2 -o sq2 --output-format csv -- python3 $B --steps 30 --warmup 5 > $D/sq2.log 2>&1 || exit 6
python3 tools/rocprof_summary.py $TAG --key $KEY --cmd "$B --steps 200 --warmup 20" || exit 7
