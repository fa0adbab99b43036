#!/bin/bash
# configs[4] tail attribution: repeated 1e6-QPS levels through the coalescer
# with the batch trace on; per level p99 / worst and the slow batches
# ([ms since start, stage-in us, enqueue us, own device us, m]).
# VARIANTS: one environment assignment per line ("RL_X=0" = default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
while IFS= read -r v; do
  i=$((i + 1))
  env $v RL_COALESCER_TRACE=200000 timeout -k 10 200 distributed-rate-limiter_amd/lib/rl_bench_e2e \
      --qps ${QPS:-1e6,1e6,1e6,1e6,1e6,1e6} --seconds 2 > gpurun_out/e2e_v$i.json 2>/dev/null || exit 1
  python3 - "$v" gpurun_out/e2e_v$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
for l in d["levels"]:
    t = l.get("trace", {})
    slow = [v for k, v in t.items() if k.startswith("slow")]
    print(sys.argv[1], l["offered_qps"], "p99", l["p99_us"], "max", max(l["max_us_by_100ms"]), "rq_max_us", l.get("max_thread_runqueue_wait_us"), "rq_sum_us", l.get("sum_thread_runqueue_wait_us"), "slow", slow[0][:3] if slow else None)
PY
done <<< "${VARIANTS:-RL_X=0}"
