set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --secondary > gpurun_out/bench_sec.json 2> gpurun_out/bench_sec.err || exit 1
