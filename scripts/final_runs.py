"""Collect one scripts/steps.sh call's bench lines into profiles/<TAG>_final_runs.txt and copy its
bench / e2e / gRPC JSON, GPU-suite and smoke outputs to profiles/ (python scripts/final_runs.py TAG "header")."""
import glob
import json
import os
import shutil
import sys

tag, header = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
out, prof = os.path.join(root, "gpurun_out"), os.path.join(root, "profiles")
lines = [f"# {l}" for l in header.splitlines()]
for f in sorted(glob.glob(os.path.join(out, f"{tag}_*.out"))):
    name = os.path.basename(f)[:-4]
    js = [x for x in open(f) if x.startswith("{")]
    if not js:
        continue
    d = json.loads(js[-1])
    if "ms_per_step" in d:
        lines.append(f"{name:14s} {d['value']:.4g} {d['unit']}  {d['ms_per_step'] * 1e3:.1f} us/step  "
                     f"{d['config'].get('workload', '')[:60]}")
open(os.path.join(prof, f"{tag}_final_runs.txt"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
for suffix, dst in (("bench", "bench.json"), ("e2e", "e2e.json"), ("grpc", "grpc.json")):
    f = os.path.join(out, f"{tag}_{suffix}.out")
    if os.path.exists(f):
        js = [x for x in open(f) if x.startswith("{")]
        if js:
            open(os.path.join(prof, f"{tag}_{dst}"), "w").write(js[-1])
for suffix, dst in (("gpu", "gpu_tests.txt"), ("smoke", "smoke.txt")):
    f = os.path.join(out, f"{tag}_{suffix}.out")
    if os.path.exists(f):
        shutil.copy(f, os.path.join(prof, f"{tag}_{dst}"))
