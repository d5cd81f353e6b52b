# One rocprofv3 PMC pass over a short bench run, step-kernel counters printed
# as per-launch means:  bash tools/gpu/pmc.sh TAG "COUNTERS" "BENCH ARGS"
set -o pipefail
TAG=$1; CTRS=$2; ARGS=$3
mkdir -p gpurun_out
export TMPDIR=/tmp
D=gpurun_out/pmc_$TAG
rm -rf $D
timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace -d $D -o p --output-format csv -- python3 bench.py --no-secondary --no-cpu-baseline --steps 20 --warmup 5 $ARGS > $D.log 2>&1 || exit 3
python3 - $D <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(float)
disp = defaultdict(set)
with open(sys.argv[1] + "/p_counter_collection.csv") as f:
    for r in csv.DictReader(f):
        if "step" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(acc):
    print(f"{k}: {acc[k] / len(disp[k]):,.0f} per launch")
PY
