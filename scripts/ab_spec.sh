#!/bin/bash
# A/B: speculative restart windows (default) vs none (RL_CH_SPEC=0 build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BARGS="--lat-batches 0" STEPS=20 bash scripts/ab.sh librl_amd_spec0.so librl_amd.so || exit 1
BARGS="--lat-batches 0 --workload tb_zipf15" STEPS=6 bash scripts/ab.sh librl_amd_spec0.so librl_amd.so || exit 1
BARGS="--lat-batches 0 --workload tb_hot" STEPS=4 bash scripts/ab.sh librl_amd_spec0.so librl_amd.so
