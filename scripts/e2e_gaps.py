#!/usr/bin/env python3
"""Attribute the configs[4] tail windows of one traced rl_bench_e2e run.

Usage: e2e_gaps.py <rocprof dir> <e2e json> <out.md>

The run is `RL_COALESCER_TRACE=... rocprofv3 --hip-trace --kernel-trace --
lib/rl_bench_e2e --qps ...`.  For every 100-ms window whose worst latency
passes 1 ms it lists what the device and the submitter did: device idle gaps
(no engine kernel running) of more than 300 us, the longest kernels, and the
longest stretch in which the coalescer's submitter thread (the thread that
launches the kernels) made no HIP call."""
import collections
import csv
import glob
import json
import os
import sys

ENGINE = ("k_small", "k_tb_chain", "k_probe", "k_replay_light")


def load(d, what):
    rows = []
    for f in glob.glob(os.path.join(d, "**", f"*{what}.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


d, ej, out = sys.argv[1:4]
ker = load(d, "kernel_trace")
api = load(d, "hip_api_trace")
e2e = json.load(open(ej))
eng = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in ker
             if any(k in r["Kernel_Name"] for k in ENGINE))
t0 = eng[0][0]
# device idle gaps between engine kernels
gaps, prev = [], None
for s, e, _ in eng:
    if prev is not None and s - prev > 300_000:
        gaps.append(((prev - t0) / 1e6, (s - prev) / 1e3))
    prev = e if prev is None else max(prev, e)
# the submitter: the thread that launches the kernels (most hipLaunchKernel / hipExtLaunchKernel calls)
launch = collections.Counter(a["Thread_Id"] for a in api if "Launch" in a["Function"])
sub = launch.most_common(1)[0][0]
calls = sorted((int(a["Start_Timestamp"]), int(a["End_Timestamp"])) for a in api if a["Thread_Id"] == sub)
silent = []
for (s0, e0), (s1, _) in zip(calls, calls[1:]):
    if s1 - e0 > 300_000 and s0 > t0:
        silent.append(((e0 - t0) / 1e6, (s1 - e0) / 1e3))
# the levels' windows: a level starts where its engine activity resumes after
# the previous level's idle time (> 10 ms of no kernels)
starts = [g[0] + g[1] / 1e3 for g in gaps if g[1] > 10_000]
lines = ["# configs[4] tail windows, attributed (round 6)", "",
         "Command: `RL_COALESCER_TRACE=200000 rocprofv3 --hip-trace --kernel-trace -- "
         "distributed-rate-limiter_amd/lib/rl_bench_e2e --qps 1e7,1e7 --seconds 2` "
         "(`scripts/e2e_gaps.py`).", "",
         f"Submitter thread (most kernel launches): {sub}.", "",
         "| level | window | worst us | device idle gaps in it (ms, us) | submitter silent (ms, us) | "
         "run-queue max us (level) |", "|---|---|---|---|---|---|"]
for li, lv in enumerate(e2e["levels"]):
    base = starts[li] if li < len(starts) else None
    for wi, w in enumerate(lv["max_us_by_100ms"]):
        if w <= 1000 or base is None:
            continue
        lo, hi = base + 100 * wi - 20, base + 100 * (wi + 1) + 20
        g = [f"{a:.1f}, {b:.0f}" for a, b in gaps if lo <= a < hi and b < 10_000]
        s = [f"{a:.1f}, {b:.0f}" for a, b in silent if lo <= a < hi]
        lines.append(f"| {li} | {wi} | {w} | {'; '.join(g) or '-'} | {'; '.join(s) or '-'} | "
                     f"{lv.get('max_thread_runqueue_wait_us')} |")
by = collections.defaultdict(list)
for s, e, n in eng:
    by[n.split("(")[0].replace("void ", "")].append((e - s) / 1e3)
lines += ["", "Longest engine kernels of the run:", "", "| kernel | launches | p50 us | max us |", "|---|---|---|---|"]
for n, v in sorted(by.items(), key=lambda kv: -max(kv[1])):
    v.sort()
    lines.append(f"| `{n}` | {len(v)} | {v[len(v) // 2]:.0f} | {v[-1]:.0f} |")
open(out, "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
