#!/usr/bin/env python3
"""Attribute the configs[4] tail: read a rocprofv3
--hip-trace --kernel-trace --memory-copy-trace run of lib/rl_bench_e2e and
report the longest HIP API calls, with the kernels and copies that ran on
the device while each one blocked.  Usage: stall_trace.py <rocprof dir> <out.json>"""
import csv
import glob
import json
import os
import sys


def load(pattern):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


d, out = sys.argv[1], sys.argv[2]
api = load(os.path.join(d, "**", "*hip_api_trace.csv"))
ker = load(os.path.join(d, "**", "*kernel_trace.csv"))
cpy = load(os.path.join(d, "**", "*memory_copy_trace.csv"))
res = {"api_calls": len(api), "kernels": len(ker), "copies": len(cpy),
       "api_columns": list(api[0].keys()) if api else [], "kernel_columns": list(ker[0].keys()) if ker else []}


def span(r):
    return int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp"))


# per function: count, total, max
by_fn = {}
for r in api:
    s, e = span(r)
    fn = col(r, "Function", "Operation")
    c = by_fn.setdefault(fn, [0, 0, 0])
    c[0] += 1
    c[1] += e - s
    c[2] = max(c[2], e - s)
res["api_by_function_us"] = {k: {"calls": v[0], "total_us": v[1] / 1e3, "max_us": v[2] / 1e3}
                             for k, v in sorted(by_fn.items(), key=lambda kv: -kv[1][2])[:25]}
dev = [(span(r), "kernel", col(r, "Kernel_Name", "Name")) for r in ker] + \
      [(span(r), "copy", col(r, "Operation", "Direction", "Name") if r else "") for r in cpy]
dev.sort()
t0 = min([span(r)[0] for r in api] + [x[0][0] for x in dev]) if api else 0
# the load phase only: calls of the per-batch functions (set-up calls such as
# stream creation are excluded)
hot = {"hipMemcpyAsync", "hipEventSynchronize", "hipLaunchKernel", "hipEventRecord", "hipStreamWaitEvent",
       "hipExtLaunchKernel", "hipEventQuery", "hipSetDevice"}
load_start = min((span(r)[0] for r in api if col(r, "Function", "Operation") == "hipMemcpyAsync"), default=0)
longest = sorted((r for r in api if col(r, "Function", "Operation") in hot and span(r)[0] > load_start + 50_000_000),
                 key=lambda r: span(r)[0] - span(r)[1])[:12]
stalls = []
for r in longest:
    s, e = span(r)
    during = [{"what": w, "name": n[:60], "start_us": (a - t0) / 1e3, "dur_us": (b - a) / 1e3}
              for (a, b), w, n in dev if b > s and a < e]
    # the device items that were longest inside the blocked interval
    during.sort(key=lambda x: -x["dur_us"])
    gaps = 0.0
    busy = sorted([(max(a, s), min(b, e)) for (a, b), _, _ in dev if b > s and a < e])
    cur = s
    for a, b in busy:
        if a > cur:
            gaps += a - cur
        cur = max(cur, b)
    gaps += max(0, e - cur)
    stalls.append({"function": col(r, "Function", "Operation"), "thread": r.get("Thread_Id"),
                   "start_us": (s - t0) / 1e3, "dur_us": (e - s) / 1e3,
                   "device_idle_us_inside": gaps / 1e3, "device_items_inside": len(during),
                   "longest_device_items_inside": during[:6]})
res["longest_api_calls"] = stalls
# the worst call's neighbourhood: every API call of every thread that overlaps
# [start - 2 ms, end + 1 ms], and the device items in the same window
if longest:
    s0, e0 = span(longest[0])
    w0, w1 = s0 - 2_000_000, e0 + 1_000_000
    near = sorted((span(r)[0], span(r)[1], r.get("Thread_Id"), col(r, "Function", "Operation")) for r in api
                  if span(r)[1] > w0 and span(r)[0] < w1)
    res["worst_window_api"] = [{"t_us": (a - t0) / 1e3, "dur_us": (b - a) / 1e3, "thread": th, "fn": fn}
                               for a, b, th, fn in near if b - a > 20_000 or fn == "hipMemcpyAsync"][:300]
    res["worst_window_device"] = [{"t_us": (a - t0) / 1e3, "dur_us": (b - a) / 1e3, "what": w, "name": n[:50]}
                                  for (a, b), w, n in dev if b > w0 and a < w1][:400]
kd = sorted(((span(r)[1] - span(r)[0], col(r, "Kernel_Name", "Name"), span(r)[0]) for r in ker), reverse=True)[:10]
res["longest_kernels"] = [{"dur_us": a / 1e3, "name": b[:60], "start_us": (c - t0) / 1e3} for a, b, c in kd]
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: res[k] for k in ("api_calls", "kernels", "copies")}))
for s in stalls[:5]:
    print(s["function"], round(s["dur_us"]), "us at", round(s["start_us"]), "device idle inside", round(s["device_idle_us_inside"]))
