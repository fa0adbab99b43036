#!/bin/bash
# neighbouring-decade serial steps vs the base build; GPU suite on the new build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/nb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/nb_tests.log
[ $rc -ge 124 ] && exit $rc
BARGS="--workload tb_zipf15 --lat-batches 0" STEPS=8 bash scripts/ab.sh librl_amd_base.so librl_amd.so librl_amd_base.so librl_amd.so || exit $?
BARGS="--lat-batches 0" STEPS=16 bash scripts/ab.sh librl_amd_base.so librl_amd.so || exit $?
BARGS="--workload tb_hot --lat-batches 0" STEPS=4 bash scripts/ab.sh librl_amd_base.so librl_amd.so || exit $?
RL_AMD_LIB=$PWD/distributed-rate-limiter_amd/lib/librl_amd_stamps.so TAG=stamps_nb BARGS="--workload tb_zipf15" STEPS=6 bash scripts/bench_brief.sh
