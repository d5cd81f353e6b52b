set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/tall.log 2>&1; echo "rc=$?" >> gpurun_out/tall.log
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/skip0.log 2>&1 || exit 1
