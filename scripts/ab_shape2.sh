#!/bin/bash
# A/B: chain shapes (producers x requests per lane) with speculative windows
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BARGS="--lat-batches 0" STEPS=20 bash scripts/ab.sh librl_amd.so librl_amd_np8k5.so librl_amd_np6k6.so librl_amd_np7k4.so || exit 1
BARGS="--lat-batches 0 --workload tb_zipf15" STEPS=6 bash scripts/ab.sh librl_amd.so librl_amd_np8k5.so librl_amd_np6k6.so librl_amd_np7k4.so
