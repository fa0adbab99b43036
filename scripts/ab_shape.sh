#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BARGS="--lat-batches 0" STEPS=16 bash scripts/ab.sh librl_amd.so librl_amd_np6k6.so librl_amd_np8k4.so librl_amd_np5k8.so librl_amd_np9k4.so
BARGS="--workload tb_zipf15 --lat-batches 0" STEPS=8 bash scripts/ab.sh librl_amd.so librl_amd_np6k6.so librl_amd_np8k4.so
