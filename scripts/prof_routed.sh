#!/bin/bash
# routed configs[3] on one GPU: kernel trace (timeline per queue) of the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-r2j_routed}
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${TAG}_trace -o run -- python3 bench.py --workload mixed --ingress routed --steps 12 --warmup 3 --no-cpu-baseline --lat-batches 0 > gpurun_out/prof/${TAG}.log 2>&1
echo rc=$?
