#!/usr/bin/env python3
"""Print the kernel timeline of one rocprofv3 --kernel-trace run (the last
few batches): start/end relative to the first kernel shown, per stream."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    name = name.replace("rl::", "")[:28]
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{name:28s} q{r.get('Queue_Id', r.get('Stream_Id', '?')):>3} {s:9.1f} {e:9.1f} {e - s:8.1f}")
