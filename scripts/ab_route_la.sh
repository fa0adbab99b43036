#!/bin/bash
# routed pipeline lookahead / depth sweep (world 1, configs[3])
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
for cfg in "2 6" "3 6" "4 8" "5 8"; do
  set -- $cfg
  RL_ROUTE_LOOKAHEAD=$1 RL_ROUTE_DEPTH=$2 timeout -k 10 200 python bench.py --workload mixed --ingress routed --steps 16 --warmup 3 --no-cpu-baseline --lat-batches 0 2>/dev/null \
    | python -c "import json,sys; d=json.load(sys.stdin); print('lookahead $1 depth $2', round(d['value']/1e6,1), d['config'].get('host_ms_per_step'))" || exit 1
done
done
