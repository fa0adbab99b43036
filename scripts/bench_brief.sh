#!/bin/bash
# One short bench run; prints value, stage ms and replay timers (for A/B sweeps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 200 python bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline ${BARGS:-} > /tmp/bb.json || exit $?
python - "${TAG:-}" <<'PY'
import json, sys
d = json.load(open("/tmp/bb.json"))
r = d["replay_detail"]
print(sys.argv[1], "| %.1f M/s" % (d["value"] / 1e6),
      {k: round(x, 3) for k, x in d["stages_ms_per_batch"].items()},
      "timers_us", [round(x / 100, 1) for x in r["stamp_cycles_longest_segment"][:6]], "rounds", r["coop_rounds"], "iters", r["coop_iters"],
      "maxr", r["stamp_cycles_longest_segment"][6], "ends", r.get("coop_ends"))
w = r.get("wave_phase_cycles", [])
if any(w):
    n = max(1, r["stamp_cycles_longest_segment"][6])
    for k in range(8):
        print("  wave", k, "cycles/round per phase", [round(x / n) for x in w[8 * k:8 * k + 8]])
PY
