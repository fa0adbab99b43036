"""Summarize A/B bench lines of one gpurun call: python scripts/abx.py TAG"""
import glob
import json
import os
import sys

tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{tag}_*.out"), key=os.path.getmtime):
    lines = [x for x in open(f) if x.startswith("{")]
    name = os.path.basename(f)[:-4]
    if not lines:
        tail = open(f).read().strip().splitlines()[-1:] or [""]
        print(f"{name:24s} {tail[0][:100]}")
        continue
    d = json.loads(lines[-1])
    if "value" not in d or "ms_per_step" not in d:
        print(f"{name:24s} (no decisions/s line)")
        continue
    rf = d.get("roofline", {})
    rd = d.get("replay_detail", {})
    print(f"{name:24s} {d['value']:.4e}  step {d['ms_per_step']*1e3:7.1f} us  replay {rf.get('launch_ms', 0)*1e3:7.1f} us"
          + (f"  xdec {rd['xdec'][:4]}" if 'xdec' in rd else "")
          + (f"  st {rd['stamps_x16'][:5]} split {rd.get('split_x16')}" if rd.get('stamps_x16', [0])[0] else ""))
