set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_rollout.py -q -x > gpurun_out/troll.log 2>&1; echo "rc=$?" >> gpurun_out/troll.log
timeout -k 10 500 python bench.py --secondary > gpurun_out/bench_sec.json 2> gpurun_out/bench_sec.err || exit 1
