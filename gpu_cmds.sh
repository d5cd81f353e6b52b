set -o pipefail
mkdir -p gpurun_out
E32=littoral-naval-warfare-marl_amd/lnw/liblnw_e32.so
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x > gpurun_out/t2.log 2>&1; echo "rc=$?" >> gpurun_out/t2.log
LNW_LIB=$E32 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x > gpurun_out/t2_32.log 2>&1; echo "rc=$?" >> gpurun_out/t2_32.log
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/skip0.log 2>&1 || exit 1
LNW_LIB=$E32 timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/e32.log 2>&1 || exit 1
LNW_LIB=$E32 LNW_PROF=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof32.log 2>&1 || exit 1
