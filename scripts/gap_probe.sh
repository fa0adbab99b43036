#!/bin/bash
# configs[1]: replay-to-replay gaps on the chain stream (kernel trace), and the
# bench with / without the timed region's replay events
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gap
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --lat-batches 0 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('timing on ', round(d['value']/1e6,1))"
  RL_BENCH_NO_TIMING=1 timeout -k 10 200 python bench.py --steps 20 --warmup 4 --no-cpu-baseline --lat-batches 0 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('timing off', round(d['value']/1e6,1))"
done
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap/trace -o run -- python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --lat-batches 0 > gpurun_out/gap/bench.log 2>&1
echo trace rc=$?
