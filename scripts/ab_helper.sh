#!/bin/bash
# replay helper kernel (k_replay_rest on its own stream) vs the base build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/helper_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/helper_tests.log
[ $rc -ge 124 ] && exit $rc
for wl in fw_uniform sw_bursty mixed tb_zipf; do
  BARGS="--workload $wl --lat-batches 0" STEPS=12 bash scripts/ab.sh librl_amd_base.so librl_amd.so || exit $?
done
BARGS="--workload tb_zipf15 --lat-batches 0" STEPS=6 bash scripts/ab.sh librl_amd_base.so librl_amd.so || exit $?
