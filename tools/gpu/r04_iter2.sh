set -o pipefail
bash tools/gpu/tests.sh "rollout or policy or torch_impl" || exit 1
bash tools/gpu/c5_trace.sh r04_c5b || exit 2
