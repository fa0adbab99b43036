#!/bin/bash
# A/B: exit step's n / config loaded during its tile's exact replay (default)
# vs loaded by the serial step (librl_amd_base.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BARGS="--lat-batches 0" STEPS=20 bash scripts/ab.sh librl_amd_base.so librl_amd.so || exit 1
BARGS="--lat-batches 0 --workload tb_zipf15" STEPS=6 bash scripts/ab.sh librl_amd_base.so librl_amd.so
