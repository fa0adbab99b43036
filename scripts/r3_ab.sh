#!/bin/bash
# routed pipeline at world 1: route tests, then depth / lookahead A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_route_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ab_tests.txt 2>&1 || { tail -20 gpurun_out/r3ab_tests.txt; exit 1; }
tail -1 gpurun_out/r3ab_tests.txt
for dl in "6 2" "8 3" "10 4" "6 2" "8 3" "10 4"; do
  set -- $dl
  export RL_ROUTE_DEPTH=$1 RL_ROUTE_LOOKAHEAD=$2
  timeout -k 10 200 python bench.py --workload mixed --ingress routed --steps 30 --warmup 3 --no-cpu-baseline --lat-batches 0 > gpurun_out/r3ab.json 2> gpurun_out/r3ab.err || { tail gpurun_out/r3ab.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r3ab.json')); print('depth=$1 L=$2', round(d['value']/1e6,1), round(d['ms_per_step'],3), json.dumps(d['config']['host_ms_per_step']))"
done
