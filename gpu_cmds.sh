set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/tall.log 2>&1; echo "rc=$?" >> gpurun_out/tall.log
LNW_FORCE_GENERIC=1 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x > gpurun_out/t2g.log 2>&1; echo "rc=$?" >> gpurun_out/t2g.log
timeout -k 10 400 python bench.py --secondary > gpurun_out/bench_sec.json 2> gpurun_out/bench_sec.err || exit 1
