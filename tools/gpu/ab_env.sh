# Interleaved A/B of one environment knob on bench.py workloads (kernel time):
#   bash tools/gpu/ab_env.sh VAR[=VALUE] ROUNDS "BENCH ARGS" ["BENCH ARGS" ...]
# each round runs every workload without and with VAR=VALUE (default 1), alternating.
set -o pipefail
VAR=${1%%=*}; VAL=${1#*=}; [ "$VAL" = "$1" ] && VAL=1; ROUNDS=$2; shift 2
mkdir -p gpurun_out
for r in $(seq "$ROUNDS"); do
  for args in "$@"; do
    for on in 0 1; do
      if [ "$on" = 1 ]; then export "$VAR"="$VAL"; else unset "$VAR"; fi
      timeout -k 10 120 python bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 $args \
        > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -15 gpurun_out/ab.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('r$r', '$VAR=$on', '$args', round(d['roofline']['kernel_ms_mean']*1e3, 2), 'us')"
    done
  done
done
