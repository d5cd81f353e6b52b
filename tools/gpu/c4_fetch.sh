# Config 4 (group kernel): FETCH_SIZE per launch under section skips of the
# diagnostics build (LNW_DEBUG_SKIP; results change, traffic is attributed by
# difference), one rocprofv3 PMC pass each:
#   bash tools/gpu/c4_fetch.sh > gpurun_out/c4_fetch.txt
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
DIAG=$PWD/littoral-naval-warfare-marl_amd/lnw/liblnw_diag.so
for b in 0 1 128 65536 65665 4096 1048576 16384 march; do
  D=gpurun_out/c4f_$b; rm -rf $D
  M=""; [ "$b" = march ] && { b=0; M=1; }
  if [ -n "$M" ]; then export LNW_GROUP_MARCH=1; else unset LNW_GROUP_MARCH; fi
  LNW_LIB=$DIAG LNW_DEBUG_SKIP=$b timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D -o p --output-format csv -- python3 bench.py --no-secondary --no-cpu-baseline --steps 20 --warmup 5 --workload config4 > $D.log 2>&1 || { echo "skip $b failed"; tail -3 $D.log; exit 3; }
  python3 - $D $b "$M" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(float); disp = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1] + "/p_counter_collection.csv")):
    if "step_group_kernel" not in r["Kernel_Name"]:
        continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp[r["Counter_Name"]].add(r["Dispatch_Id"])
f = acc["FETCH_SIZE"] / len(disp["FETCH_SIZE"]) * 1024
print(f"skip {sys.argv[2]:>8}{' (LOS by march)' if sys.argv[3] else ''}: 2xFETCH {2 * f / 1e6:7.2f} MB per launch")
PY
done
