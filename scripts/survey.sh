#!/bin/bash
# GPU-box run: one short bench line per workload (and ingress), for the
# per-workload table in DESIGN.md.  Output: gpurun_out/survey/<name>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/survey
RUNS=${RUNS:-"tb_zipf: tb_zipf15: tb_hot: fw_uniform: sw_bursty: mixed: mixed:routed tb_zipf:routed"}
for r in $RUNS; do
  wl=${r%%:*}; ing=${r#*:}
  name=$wl${ing:+_$ing}
  extra=""; [ -n "$ing" ] && extra="--ingress $ing"
  timeout -k 10 240 python bench.py --workload $wl $extra --steps ${STEPS:-12} --warmup 3 --no-cpu-baseline \
      --lat-batches 0 ${BARGS:-} > gpurun_out/survey/$name.json 2> gpurun_out/survey/$name.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 gpurun_out/survey/$name.err; [ $rc -ge 124 ] && exit $rc; continue; fi
  python - "$name" gpurun_out/survey/$name.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
st = d.get("stages_ms_per_batch") or {}
print("%-18s %8.1f M/s  ms/step %.3f  stages %s  frac %.4f" % (sys.argv[1], d["value"] / 1e6, d["ms_per_step"],
      {k: round(v, 3) for k, v in st.items()}, d["roofline"]["frac"]))
PY
done
exit 0
