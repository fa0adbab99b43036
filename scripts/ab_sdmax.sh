#!/bin/bash
# A/B: speculative windows with a state bound from the guess (default) vs DEC_HI (base)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BARGS="--lat-batches 0" STEPS=20 bash scripts/ab.sh librl_amd_base.so librl_amd.so || exit 1
BARGS="--lat-batches 0 --workload tb_zipf15" STEPS=6 bash scripts/ab.sh librl_amd_base.so librl_amd.so
