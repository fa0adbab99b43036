#!/bin/bash
# A/B: strtod quotient by corrected product (default) vs IEEE division
# (RL_STEP_MK=0 build), configs[1] and Zipf 1.5 / one hot key
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BARGS="--lat-batches 0" STEPS=20 bash scripts/ab.sh librl_amd_mk0.so librl_amd.so || exit 1
BARGS="--lat-batches 0 --workload tb_zipf15" STEPS=6 bash scripts/ab.sh librl_amd_mk0.so librl_amd.so || exit 1
BARGS="--lat-batches 0 --workload tb_hot" STEPS=4 bash scripts/ab.sh librl_amd_mk0.so librl_amd.so
