set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_kt.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof_fetch -o fetch --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/prof_write -o write --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_write.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d gpurun_out/prof_sq -o sq --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_sq.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/prof_sq2 -o sq2 --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_sq2.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --secondary > gpurun_out/bench_sec.json 2> gpurun_out/bench_sec.err || exit 7
