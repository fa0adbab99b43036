#!/bin/bash
# GPU suite, then A/B of the current build against librl_amd_base.so (HEAD
# before the change) on the uniform workloads and configs[1]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=tests bash scripts/gpu_check.sh || exit $?
grep -q " passed" gpurun_out/gpu_tests.log && ! grep -qE "[0-9]+ failed|ERROR" gpurun_out/gpu_tests.log || { echo TESTS-FAILED; exit 1; }
for wl in mixed fw_uniform sw_bursty tb_zipf; do
  BARGS="--workload $wl --lat-batches 0" STEPS=12 bash scripts/ab.sh librl_amd_base.so librl_amd.so || exit $?
done
for v in librl_amd_base.so librl_amd.so; do
  RL_AMD_LIB=$PWD/distributed-rate-limiter_amd/lib/$v timeout -k 10 200 python bench.py --workload mixed --ingress routed --steps 12 --warmup 3 --no-cpu-baseline --lat-batches 0 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('routed $v', round(d['value']/1e6,1))" || exit 1
done
