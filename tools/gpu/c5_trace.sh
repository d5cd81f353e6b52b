# rocprofv3 kernel trace + stats of config 5 (tools/config5_profile.py) into
# gpurun_out/$1 (default c5); the summary: python tools/rocprof_summary.py TAG --trace-only ...
set -o pipefail
TAG=${1:-c5}
export TMPDIR=/tmp
mkdir -p gpurun_out
D=gpurun_out/$TAG
rm -rf $D; mkdir -p $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- python3 tools/config5_profile.py > $D/kt.log 2>&1 || { tail -20 $D/kt.log; exit 2; }
tail -1 $D/kt.log
python3 - "$D" <<'PY'
import csv, sys, os
d = sys.argv[1]
rows = list(csv.DictReader(open(os.path.join(d, "kt", "kt_kernel_stats.csv"))))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{r["Name"][:90]:90s} calls {r["Calls"]:>7s} mean {float(r["AverageNs"])/1e3:9.2f} us total {float(r["TotalDurationNs"])/1e6:9.2f} ms')
PY
