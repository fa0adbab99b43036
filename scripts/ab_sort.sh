#!/bin/bash
# A/B of the grouping kernels' tile sizes (make variant builds) on the
# uniform workloads, local and routed ingress
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BARGS="--workload mixed --lat-batches 0" bash scripts/ab.sh librl_amd.so librl_amd_si8.so librl_amd_si4.so librl_amd_si8g8.so || exit $?
BARGS="--workload fw_uniform --lat-batches 0" STEPS=12 bash scripts/ab.sh librl_amd.so librl_amd_si8.so librl_amd_si4.so || exit $?
for v in librl_amd.so librl_amd_si8.so librl_amd_si4.so; do
  RL_AMD_LIB=$PWD/distributed-rate-limiter_amd/lib/$v timeout -k 10 200 python bench.py --workload mixed --ingress routed --steps 12 --warmup 3 --no-cpu-baseline --lat-batches 0 \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('routed $v', round(d['value']/1e6,1))" || exit 1
done
