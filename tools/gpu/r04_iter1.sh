set -o pipefail
bash tools/gpu/tests.sh "rollout or policy or torch_impl" || exit 1
timeout -k 10 400 python tools/config5_profile.py > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -20 gpurun_out/c5.err; exit 2; }
cat gpurun_out/c5.json
bash tools/gpu/ab_env.sh LNW_NO_XCD_REMAP 3 "--global-envs 8192" "--global-envs 4096" "--workload config4" ""
