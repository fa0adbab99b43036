#!/bin/bash
# exact-step variants: GPU suite on the combined variant, then A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RL_AMD_LIB_TEST=$PWD/distributed-rate-limiter_amd/lib/librl_amd_divrint.so
RL_AMD_LIB=$RL_AMD_LIB_TEST timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/step_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/step_tests.log
BARGS="--lat-batches 0" STEPS=16 bash scripts/ab.sh librl_amd.so librl_amd_div.so librl_amd_rint.so librl_amd_divrint.so || exit $?
BARGS="--workload tb_zipf15 --lat-batches 0" STEPS=8 bash scripts/ab.sh librl_amd.so librl_amd_divrint.so || exit $?
