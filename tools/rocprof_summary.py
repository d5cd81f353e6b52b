#!/usr/bin/env python3
"""Summarise the rocprofv3 runs of tools/gpu/prof.sh into profiles/<tag>_*.

Reads gpurun_out/<tag>/kt (kernel trace + stats) and the separate --pmc passes
(fetch, write, sq, sq2), writes
  profiles/<tag>_kernel_stats.csv   (copy of rocprofv3's kernel_stats)
  profiles/<tag>_rocprof.md         (stats table, step-kernel PMC, roofline)
and records the step kernel's per-launch HBM bytes 2 x FETCH_SIZE + WRITE_SIZE
(KB -> B; gfx950 FETCH_SIZE counts half the bytes of 16-B/lane streamed reads,
MI355X_MICROARCH.md § HBM) in profiles/traffic.json under KEY, together with
the SHA-256 of the liblnw.so measured (bench.py reports the figure only for
that same library).

usage: python tools/rocprof_summary.py TAG --key reference_e65536_los0_mv0 --cmd "..."
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
sys.path.insert(0, ROOT)
PROF = os.path.join(ROOT, "profiles")


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    if n.startswith("step_kernel") and ">" in n:
        return n[: n.index(">") + 1]
    return n.split("(")[0]


def counters(d, stem):
    path = os.path.join(OUT, d, f"{stem}_counter_collection.csv")
    acc = defaultdict(list)
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if "step_kernel" not in r["Kernel_Name"] and "step_group_kernel" not in r["Kernel_Name"]:
                continue
            acc[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    per = defaultdict(list)
    for (disp, name), v in acc.items():
        per[name].append(sum(v))
    return {k: sum(v) / len(v) for k, v in per.items()}


def trace_only(tag, cmd, steps):
    """profiles/<tag>_rocprof.md from a --kernel-trace --stats run alone: every
    kernel's calls, mean and total time, and (given the number of env steps the
    command ran) the time per step of each kernel family."""
    d = os.path.join(OUT, tag)
    stats = os.path.join(d, "kt", "kt_kernel_stats.csv")
    shutil.copy(stats, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# rocprofv3 --kernel-trace --stats: {cmd}", "",
             "| kernel | calls | avg us | total ms | % | us per env step |", "|---|---|---|---|---|---|"]
    for r in rows:
        t = float(r["TotalDurationNs"])
        per = f"{t / 1e3 / steps:.1f}" if steps else "-"
        lines.append(f"| {short(r['Name'])[:90]} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{t / 1e6:.2f} | {100 * t / tot:.1f} | {per} |")
    if steps:
        lines += ["", f"GPU kernel time per env step (all kernels): {tot / 1e3 / steps:.1f} us over {steps} steps"]
    open(os.path.join(PROF, f"{tag}_rocprof.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


C5_FAMILIES = (("observe", "observe_kernel"), ("policy", "policy_act_kernel"), ("step", "step_kernel"),
                ("post", "rollout_post_kernel"))


def family_counters(d, stem):
    """Per-launch mean of every counter of a --pmc pass, per config-5 kernel family."""
    path = os.path.join(OUT, d, f"{stem}_counter_collection.csv")
    if not os.path.exists(path):
        return {}
    acc = defaultdict(float)
    disp = defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            fam = next((k for k, sub in C5_FAMILIES if sub in r["Kernel_Name"]), None)
            if fam is None:
                continue
            acc[(fam, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[(fam, r["Counter_Name"])].add(r["Dispatch_Id"])
    out = defaultdict(dict)
    for (fam, name), v in acc.items():
        out[fam][name] = v / len(disp[(fam, name)])
    return out


def config5(tag, cmd, envs):
    """profiles/<tag>_rocprof.md for config 5: each of the four launches of a
    rollout step with its mean time, algorithmic bytes (bench.config5_bytes),
    PMC traffic 2 x FETCH_SIZE + WRITE_SIZE and SQ counters."""
    import bench
    d = os.path.join(OUT, tag)
    stats = os.path.join(d, "kt", "kt_kernel_stats.csv")
    shutil.copy(stats, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    avg = {}
    for fam, sub in C5_FAMILIES:
        for r in rows:
            if sub in r["Name"] and fam not in avg:
                avg[fam] = (float(r["AverageNs"]) / 1e3, short(r["Name"]), int(r["Calls"]))
    pmc = defaultdict(dict)
    for sub in ("fetch", "write", "sq", "sq2"):
        for fam, cs in family_counters(os.path.join(tag, sub), sub).items():
            pmc[fam].update(cs)
    B = bench.config5_bytes()
    lines = [f"# rocprofv3, config 5: {cmd}", "",
             f"{envs} envs (4v4, blue actor, scripted red) per launch; algorithmic bytes per env-step from "
             "bench.config5_bytes; PMC per launch (mean), separate --pmc passes; traffic = 2 x FETCH_SIZE + "
             "WRITE_SIZE (gfx950 correction).", "",
             "| launch | kernel | calls | avg us | alg B/env-step | alg MB | frac of 8 TB/s | PMC MB | PMC/alg "
             "| WAIT_ANY/WAVE_CYC | VALU/WAVE_CYC |",
             "|---|---|---|---|---|---|---|---|---|---|---|"]
    tot_t = tot_b = 0.0
    for fam, _ in C5_FAMILIES:
        if fam not in avg:
            continue
        t, name, calls = avg[fam]
        alg = B[fam] * envs
        tot_t += t
        tot_b += alg
        p = pmc.get(fam, {})
        traf = (2 * p["FETCH_SIZE"] + p["WRITE_SIZE"]) * 1024 if "FETCH_SIZE" in p and "WRITE_SIZE" in p else None
        wc = p.get("SQ_WAVE_CYCLES")
        wait = f"{p['SQ_WAIT_ANY'] / wc:.2f}" if wc and "SQ_WAIT_ANY" in p else "-"
        valu = f"{p['SQ_ACTIVE_INST_VALU'] / wc:.2f}" if wc and "SQ_ACTIVE_INST_VALU" in p else "-"
        lines.append(f"| {fam} | {name[:48]} | {calls} | {t:.1f} | {B[fam]} | {alg / 1e6:.1f} | "
                     f"{alg / (t * 1e-6) / 8e12:.3f} | {'-' if traf is None else f'{traf / 1e6:.1f}'} | "
                     f"{'-' if traf is None else f'{traf / alg:.2f}'} | {wait} | {valu} |")
    lines += ["", f"Step (four launches): {tot_t:.1f} us of kernel time, {tot_b / 1e6:.1f} MB algorithmic -> "
                  f"{tot_b / (tot_t * 1e-6) / 8e12:.3f} of 8 TB/s", "", "Raw counters per launch:"]
    for fam, _ in C5_FAMILIES:
        for k in sorted(pmc.get(fam, {})):
            lines.append(f"- {fam} {k}: {pmc[fam][k]:,.0f}")
    open(os.path.join(PROF, f"{tag}_rocprof.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


def main():
    import hashlib
    import bench
    tag = sys.argv[1]
    if "--config5" in sys.argv:
        return config5(tag, sys.argv[sys.argv.index("--cmd") + 1] if "--cmd" in sys.argv else "",
                       int(sys.argv[sys.argv.index("--envs") + 1]) if "--envs" in sys.argv else 32768)
    key = sys.argv[sys.argv.index("--key") + 1] if "--key" in sys.argv else None
    if key is None:  # kernel trace only (config 5): the stats table and the per-step split
        return trace_only(tag, sys.argv[sys.argv.index("--cmd") + 1] if "--cmd" in sys.argv else "",
                          int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 0)
    cmd = sys.argv[sys.argv.index("--cmd") + 1] if "--cmd" in sys.argv else "bench.py"
    d = os.path.join(OUT, tag)
    stats = os.path.join(d, "kt", "kt_kernel_stats.csv")
    shutil.copy(stats, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    lines = [f"# rocprofv3 --kernel-trace --stats: python3 {cmd}", "",
             "| kernel | calls | avg us | min us | max us | % |", "|---|---|---|---|---|---|"]
    step_avg, step_name = None, None
    for r in rows:
        avg = float(r["AverageNs"]) / 1e3
        lines.append(f"| {short(r['Name'])} | {r['Calls']} | {avg:.1f} | {float(r['MinNs']) / 1e3:.1f} | "
                     f"{float(r['MaxNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
        if ("step_kernel" in r["Name"] or "step_group_kernel" in r["Name"]) and step_avg is None:
            step_avg, step_name = avg, short(r["Name"])
    pmc = {}
    for sub in ("fetch", "write", "sq", "sq2"):
        pmc.update(counters(os.path.join(tag, sub), sub))
    lines += ["", f"## {step_name} PMC (per launch, mean over launches; separate --pmc passes)", ""]
    for k in sorted(pmc):
        lines.append(f"- {k}: {pmc[k]:,.0f}")
    parts = key.split("_")
    E = int(parts[1][1:])
    nb, nr = (8, 10) if parts[0] == "config4" else (4, 4)
    B = bench.algorithmic_bytes(nb, nr, quiet=parts[0] == "reference" and parts[2] == "los0")
    alg = B * E
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        fetch, write = pmc["FETCH_SIZE"] * 1024, pmc["WRITE_SIZE"] * 1024
        traffic = 2 * fetch + write
        lines += ["", f"HBM traffic per launch = 2 x FETCH_SIZE + WRITE_SIZE = {traffic / 1e6:.2f} MB "
                      f"(FETCH {fetch / 1e6:.2f} MB raw, WRITE {write / 1e6:.2f} MB); algorithmic "
                      f"{alg / 1e6:.2f} MB ({B} B/env-step x {E}); ratio {traffic / alg:.3f}"]
        tf = os.path.join(PROF, "traffic.json")
        tj = json.load(open(tf)) if os.path.exists(tf) else {}
        sys.path.insert(0, os.path.join(ROOT, "littoral-naval-warfare-marl_amd"))
        from lnw.build import source_digest
        sha = source_digest()
        if tj.get("src_sha256") != sha:
            tj = {"src_sha256": sha, "launch_bytes": {}}
        tj.setdefault("launch_bytes", {})[key] = traffic
        tj["_note"] = ("HBM bytes per step_kernel launch = 2*FETCH_SIZE + WRITE_SIZE from rocprofv3 PMC, "
                       "for the liblnw.so built from the sources and flags with this SHA-256 "
                       "(lnw.build.source_digest; tools/gpu/prof.sh, profiles/*_rocprof.md)")
        json.dump(tj, open(tf, "w"), indent=1)
    if "SQ_WAVES" in pmc and "SQ_INSTS_VALU" in pmc:
        w = pmc["SQ_WAVES"]
        lines.append(f"VALU instructions per wave: {pmc['SQ_INSTS_VALU'] / w:,.0f}; LDS instructions per wave: "
                     f"{pmc.get('SQ_INSTS_LDS', 0) / w:,.0f} ({w:,.0f} waves)")
        if "SQ_WAVE_CYCLES" in pmc and "SQ_WAIT_INST_ANY" in pmc:
            lines.append(f"SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES = {pmc['SQ_WAIT_INST_ANY'] / pmc['SQ_WAVE_CYCLES']:.2f}; "
                         f"SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES = "
                         f"{pmc.get('SQ_ACTIVE_INST_VALU', 0) / pmc['SQ_WAVE_CYCLES']:.2f}")
    if step_avg:
        lines.append(f"{step_name} average duration {step_avg:.1f} us -> {alg / (step_avg * 1e-6) / 1e9:.0f} GB/s "
                     f"algorithmic = {alg / (step_avg * 1e-6) / 8e12:.3f} of 8 TB/s")
    open(os.path.join(PROF, f"{tag}_rocprof.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
