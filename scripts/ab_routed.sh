#!/bin/bash
# A/B of the routed pipeline (bench.py --ingress routed) over environment
# variants, one per line of $VARIANTS; prints decisions/s and host ms per step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
while IFS= read -r v; do
  env $v RL_ROUTE_PROFILE=1 timeout -k 10 300 python bench.py --ingress routed --workload ${WL:-mixed} --steps 20 --warmup 3 \
      --no-cpu-baseline > /tmp/rt.json 2>/dev/null || exit 1
  python3 - "$v" <<'PY'
import json, sys
d = json.loads(open("/tmp/rt.json").read().strip().splitlines()[-1])
h = d["config"]["host_ms_per_step"]
print(f"{sys.argv[1]:40s} {d['value']/1e9:.3f}e9 {d['ms_per_step']:.3f} ms", {k: round(v, 3) for k, v in h.items()})
PY
done <<< "${VARIANTS:-RL_X=0}"
