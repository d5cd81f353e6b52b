set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/t_all.log 2>&1; echo "rc=$?" >> gpurun_out/t_all.log
