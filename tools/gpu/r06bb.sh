# round 6 final evidence, part B: rocprofv3 evidence of melee, config 4 and config 5
# (prof_all.sh part 2), then the default bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/prof_all.sh r06 2 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r06bb.json 2> gpurun_out/bench_r06bb.err
rc=$?; tail -c 300 gpurun_out/bench_r06bb.json; exit $rc
