# round 4, fifth final pass (the split paths with the analytics logs on too): GPU
# suite first (analytics replays through the contact variant), profiles for the
# headline (traffic.json keyed to the current sources) and melee, then the
# round-end check
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k analytics > gpurun_out/t23.log 2>&1 || { tail -40 gpurun_out/t23.log; exit 1; }
tail -1 gpurun_out/t23.log
bash tools/gpu/prof.sh r04_headline reference_e65536_los0_mv0 "" || exit 2
bash tools/gpu/prof.sh r04_melee melee_e65536_los0_mv0 "--spawns melee" || exit 3
bash tools/gpu/final.sh || exit 4
