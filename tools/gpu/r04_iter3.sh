set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python tools/policy_probe.py littoral-naval-warfare-marl_amd/lnw/liblnw.so tools/probe/actor_base.so tools/probe/actor_NOCONV.so tools/probe/actor_NOMLP.so || exit 1
bash tools/gpu/tests.sh "rollout or policy or torch_impl" || exit 2
bash tools/gpu/timeline.sh sh8192 "--global-envs 8192" || exit 3
bash tools/gpu/timeline.sh sh4096 "--global-envs 4096" || exit 4
D=gpurun_out/r04_sh8192; rm -rf $D; mkdir -p $D
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace -d $D/$C -o $C --output-format csv -- python3 bench.py --no-secondary --no-cpu-baseline --global-envs 8192 --steps 30 --warmup 5 > $D/$C.log 2>&1 || exit 5
done
python3 - <<'PY'
import csv, glob
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/r04_sh8192/{c}/**/*counter_collection.csv", recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Kernel_Name"]:
            vals.setdefault(r["Dispatch_Id"], 0.0)
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = sorted(vals.values())
    print(c, "per launch (KB) median", v[len(v)//2], "n", len(v))
PY
