#!/bin/bash
# routed pipeline: merge on the batch stream (default) vs on the request stream
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_route_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/route_tests.log 2>&1
echo "route tests rc=$?"; tail -2 gpurun_out/route_tests.log
for rep in 1 2; do
for v in "" "RL_ROUTE_MERGE_ON_R=1"; do
  for wl in mixed tb_zipf; do
  env $v timeout -k 10 200 python bench.py --workload $wl --ingress routed --steps 16 --warmup 3 --no-cpu-baseline --lat-batches 0 2>/dev/null \
    | python -c "import json,sys; d=json.load(sys.stdin); print('$wl ${v:-merge_on_S}', round(d['value']/1e6,1), d['config'].get('host_ms_per_step'))" || exit 1
  done
done
done
