#!/usr/bin/env python3
"""Summarise the rocprofv3 runs of tools/gpu/prof_r01.sh into profiles/<tag>_*.

Reads gpurun_out/prof_kt (kernel trace + stats) and the separate --pmc passes
(prof_fetch, prof_write, prof_sq, prof_sq2), writes
  profiles/<tag>_kernel_stats.csv   (copy of rocprofv3's kernel_stats)
  profiles/<tag>_step_kernel_rocprof.md
and updates profiles/traffic.json with the step kernel's per-launch HBM bytes:
2 x FETCH_SIZE + WRITE_SIZE (KB -> B; gfx950 FETCH_SIZE counts half the bytes
of 16-B/lane streamed reads, MI355X_MICROARCH.md § HBM).

usage: python tools/rocprof_summary.py TAG [--key reference_e65536_los0_mv0]
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    if n.startswith("step_kernel"):
        return n[: n.index(">") + 1]
    return n.split("(")[0]


def counters(d, stem):
    path = os.path.join(OUT, d, f"{stem}_counter_collection.csv")
    acc = defaultdict(list)
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if "step_kernel" not in r["Kernel_Name"]:
                continue
            acc[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    per = defaultdict(list)
    for (disp, name), v in acc.items():
        per[name].append(sum(v))
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    tag = sys.argv[1]
    key = "reference_e65536_los0_mv0"
    if "--key" in sys.argv:
        key = sys.argv[sys.argv.index("--key") + 1]
    stats = os.path.join(OUT, "prof_kt", "kt_kernel_stats.csv")
    shutil.copy(stats, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    lines = [f"# rocprofv3 --kernel-trace --stats: python3 bench.py --steps 200 --warmup 20 "
             f"--no-cpu-baseline ({tag})", "",
             "| kernel | calls | avg us | min us | max us | % |", "|---|---|---|---|---|---|"]
    step_avg = None
    for r in rows:
        avg = float(r["AverageNs"]) / 1e3
        lines.append(f"| {short(r['Name'])} | {r['Calls']} | {avg:.1f} | {float(r['MinNs']) / 1e3:.1f} | "
                     f"{float(r['MaxNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
        if "step_kernel" in r["Name"] and step_avg is None:
            step_avg = avg
    pmc = {}
    for d, stem in (("prof_fetch", "fetch"), ("prof_write", "write"), ("prof_sq", "sq"), ("prof_sq2", "sq2")):
        pmc.update(counters(d, stem))
    lines += ["", "## step_kernel PMC (per launch, mean over launches; separate --pmc passes)", ""]
    for k in sorted(pmc):
        lines.append(f"- {k}: {pmc[k]:,.0f}")
    E = 65536
    alg = 2864 * E
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        fetch, write = pmc["FETCH_SIZE"] * 1024, pmc["WRITE_SIZE"] * 1024
        traffic = 2 * fetch + write
        lines += ["", f"HBM traffic per launch = 2 x FETCH_SIZE + WRITE_SIZE = {traffic / 1e6:.1f} MB "
                      f"(FETCH {fetch / 1e6:.1f} MB raw, WRITE {write / 1e6:.1f} MB); algorithmic "
                      f"{alg / 1e6:.1f} MB (2864 B/env-step x {E})"]
        tf = os.path.join(PROF, "traffic.json")
        tj = json.load(open(tf)) if os.path.exists(tf) else {}
        tj[key] = traffic
        tj["_note"] = ("HBM bytes per step_kernel launch = 2*FETCH_SIZE + WRITE_SIZE from rocprofv3 PMC "
                       f"(profiles/{tag}_step_kernel_rocprof.md)")
        json.dump(tj, open(tf, "w"), indent=1)
    if "SQ_WAVES" in pmc and "SQ_INSTS_VALU" in pmc:
        w = pmc["SQ_WAVES"]
        lines.append(f"VALU instructions per wave: {pmc['SQ_INSTS_VALU'] / w:,.0f}; LDS instructions per wave: "
                     f"{pmc.get('SQ_INSTS_LDS', 0) / w:,.0f} ({w:,.0f} waves: 2 per workgroup)")
    if step_avg:
        lines.append(f"step_kernel average duration {step_avg:.1f} us -> {alg / (step_avg * 1e-6) / 1e9:.0f} GB/s "
                     "algorithmic")
    open(os.path.join(PROF, f"{tag}_step_kernel_rocprof.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
