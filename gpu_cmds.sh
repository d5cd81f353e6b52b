set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/tgpu.log 2>&1 || { tail -30 gpurun_out/tgpu.log; exit 1; }
tail -3 gpurun_out/tgpu.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 2
cat gpurun_out/bench.json
LNW_PROF=1 timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/prof.err || exit 3
grep "lnw prof" gpurun_out/prof.err | tail -1
