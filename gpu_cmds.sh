set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x > gpurun_out/t2.log 2>&1; echo "rc=$?" >> gpurun_out/t2.log
for k in 0 1; do LNW_PROF=1 LNW_DEBUG_SKIP=$k timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof$k.log 2>&1 || exit 1; done
timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/skip0.log 2>&1
