# GPU test pass only: pytest -m gpu (optionally -k EXPR as $1), then smoke()
set -o pipefail
mkdir -p gpurun_out
K=()
[ -n "$1" ] && K=(-k "$1")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > gpurun_out/tgpu.log 2>&1 || { tail -40 gpurun_out/tgpu.log; exit 1; }
tail -3 gpurun_out/tgpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
