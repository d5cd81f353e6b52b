set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_rollout.py -q -x > gpurun_out/troll.log 2>&1; echo "rc=$?" >> gpurun_out/troll.log
timeout -k 10 300 python tools/rollout_probe.py > gpurun_out/roll.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_roll -o roll --output-format csv -- python3 tools/rollout_probe.py > gpurun_out/prof_roll.log 2>&1 || exit 1
cp $(find /tmp/prof_roll -name "*kernel_stats.csv" | head -n 1) gpurun_out/roll_kernel_stats.csv
