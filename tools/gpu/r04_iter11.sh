# round 4, iteration 11: policy strided input, bf16x3 MLP, rollout vs torch
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "policy_act or obs_options or torch_impl" > gpurun_out/t11.log 2>&1
grep -E "PASS|FAIL|Error|assert|Mismatch|Greatest" gpurun_out/t11.log | head -40
timeout -k 10 100 python tools/policy_probe.py littoral-naval-warfare-marl_amd/lnw/liblnw.so tools/probe/actor_base.so tools/probe/actor_NOMLP.so || exit 2
