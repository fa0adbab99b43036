#!/bin/bash
# A/B: an idle wave on the chain's SIMD (RL_CH_IDLE) against the base build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BARGS="--lat-batches 0" STEPS=12 bash scripts/ab.sh librl_amd_base.so librl_amd_idle.so librl_amd_l8.so || exit $?
BARGS="--workload tb_zipf15 --lat-batches 0" STEPS=8 bash scripts/ab.sh librl_amd_base.so librl_amd_idle.so || exit $?
RL_AMD_LIB=$PWD/distributed-rate-limiter_amd/lib/librl_amd_idle_stamps.so TAG=stamps_idle bash scripts/bench_brief.sh
