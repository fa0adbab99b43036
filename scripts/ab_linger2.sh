#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V="librl_amd.so librl_amd_l8.so librl_amd_l16.so librl_amd_l32s128.so"
BARGS="--workload tb_zipf15 --lat-batches 0" STEPS=8 bash scripts/ab.sh $V || exit $?
BARGS="--lat-batches 0" STEPS=16 bash scripts/ab.sh $V || exit $?
BARGS="--workload tb_hot --lat-batches 0" STEPS=4 bash scripts/ab.sh librl_amd.so librl_amd_l16.so || exit $?
