#!/usr/bin/env python3
"""Summarize one scripts/profile.sh run (gpurun_out/prof/<TAG>_*) into
profiles/<TAG>_summary.md: rocprofv3 kernel stats plus per-launch HBM bytes
from the FETCH_SIZE / WRITE_SIZE passes.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads, so
the corrected read traffic is 2 x FETCH_SIZE (an upper bound for the narrow,
random accesses of the table probes, whose width is uncalibrated).
"""
import collections
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
src = os.path.join(root, "gpurun_out", "prof")
dst = os.path.join(root, "profiles")
os.makedirs(dst, exist_ok=True)


def short(name):
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    return name.replace("void ", "").replace("rl::", "")


stats = list(csv.DictReader(open(os.path.join(src, f"{tag}_trace", "run_kernel_stats.csv"))))
shutil.copy(os.path.join(src, f"{tag}_trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
pmc = collections.defaultdict(list)
for kind in ("fetch", "write"):
    p = os.path.join(src, f"{tag}_{kind}", "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        pmc[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))

lines = [f"# rocprofv3 summary: {tag}", "",
         os.environ.get("PROF_CMD") or ("Command: `scripts/profile.sh` (bench.py, " + os.environ.get("BARGS", "--steps 10 --warmup 2") + ")"), "",
         "| kernel | calls | avg us | % | FETCH_SIZE KiB/launch | 2xFETCH MB | WRITE_SIZE MB |",
         "|---|---|---|---|---|---|---|"]
for r in stats:
    k = short(r["Name"])
    f = pmc.get((k, "FETCH_SIZE"))
    w = pmc.get((k, "WRITE_SIZE"))
    fa = sum(f) / len(f) if f else None
    wa = sum(w) / len(w) if w else None
    lines.append(f"| {k} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} | "
                 f"{'' if fa is None else f'{fa:.0f}'} | {'' if fa is None else f'{2 * fa * 1024 / 1e6:.2f}'} | "
                 f"{'' if wa is None else f'{wa * 1024 / 1e6:.2f}'} |")
lines += ["", "2xFETCH: gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM);",
          "it is an upper bound for the narrow, random reads (table probes, gathers), whose width is uncalibrated.",
          "Infinity-Cache hits are counted as fetches (not excluded)."]
open(os.path.join(dst, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
# per-launch corrected HBM bytes per kernel, read by bench.py (roofline.traffic)
traffic = {}
for r in stats:
    k = short(r["Name"])
    f, w = pmc.get((k, "FETCH_SIZE")), pmc.get((k, "WRITE_SIZE"))
    if f and w:
        traffic[k] = {"bytes_per_launch": 2 * sum(f) / len(f) * 1024 + sum(w) / len(w) * 1024,
                      "fetch_x2_bytes": 2 * sum(f) / len(f) * 1024, "write_bytes": sum(w) / len(w) * 1024,
                      "avg_ns": float(r["AverageNs"])}
if traffic:   # a trace-only run (NO_PMC) keeps the last PMC passes' numbers
    # profiles/traffic.json feeds bench.py's roofline: only bench.py profiles write it
    name = "traffic.json" if not os.environ.get("PROF_CMD") else tag + "_traffic.json"
    import subprocess
    rev = subprocess.run(["git", "-C", root, "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    json.dump({"tag": tag, "workload": os.environ.get("WORKLOAD", "tb_zipf"), "build": rev, "kernels": traffic},
              open(os.path.join(dst, name), "w"), indent=1)
