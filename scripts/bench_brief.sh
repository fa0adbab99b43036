#!/bin/bash
# One short bench run; prints value, stage ms and chain counters (for A/B sweeps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 200 python bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline ${BARGS:-} > /tmp/bb.json || exit $?
python - "${TAG:-}" <<'PY'
import json, sys
d = json.load(open("/tmp/bb.json"))
r = d["replay_detail"]
print(sys.argv[1], "| %.1f M/s" % (d["value"] / 1e6),
      {k: round(x, 3) for k, x in d["stages_ms_per_batch"].items()},
      "longest_us", round(r["stamp_cycles_longest_segment"][0] / 100, 1), "rounds", r["coop_rounds"],
      "iters", r["coop_iters"], "maxr", r["stamp_cycles_longest_segment"][6],
      "ends", r.get("round_ends_full_stop_partial_first"), "exact", r.get("exact_tiles"), "serial", r.get("serial_steps"), "timeline", r.get("replay_timeline_us"))
st = r.get("stamps_x16")
if st and any(st):
    print("  chain [full, stop, serial, barrier]", st[0:4], " producer [work,-,-,barrier]", st[4:8], " loader", st[8:12], " hot: near cyc/entries/iters", st[12], [int(x) for x in r.get("near_hot", [])], "setup", r.get("near_setup_x16"), "exact", r.get("exact_hot_x16"), " hw_id", r.get("hw_id"))
PY
