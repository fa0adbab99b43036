#!/bin/bash
# routed pipeline: count exchange on its own group/stream (default) vs shared with the records
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
for v in "" "RL_ROUTE_CNT_SHARED=1"; do
  for wl in mixed tb_zipf; do
  env $v timeout -k 10 200 python bench.py --workload $wl --ingress routed --steps 16 --warmup 3 --no-cpu-baseline --lat-batches 0 2>/dev/null \
    | python -c "import json,sys; d=json.load(sys.stdin); print('$wl ${v:-cnt_own}', round(d['value']/1e6,1), d['config'].get('host_ms_per_step'))" || exit 1
  done
done
done
