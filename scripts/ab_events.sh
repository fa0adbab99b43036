#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BARGS="--lat-batches 0" STEPS=20 bash scripts/ab.sh librl_amd_base.so librl_amd.so librl_amd_base.so librl_amd.so
