set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -x -k "episode or shard" > gpurun_out/t2.log 2>&1; echo "rc=$?" >> gpurun_out/t2.log
LNW_FORCE_GENERIC=1 timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -x -k "episode or shard" > gpurun_out/t2g.log 2>&1; echo "rc=$?" >> gpurun_out/t2g.log
for k in 0 1 2 4; do LNW_DEBUG_SKIP=$k timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/skip$k.log 2>&1 || exit 1; done
LNW_FORCE_GENERIC=1 timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/gen.log 2>&1 || exit 1
