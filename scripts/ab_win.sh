#!/bin/bash
# window-membership range check vs the base build; GPU suite on the new build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/win_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/win_tests.log
[ $rc -ge 124 ] && exit $rc
for wl in fw_uniform sw_bursty mixed; do
  BARGS="--workload $wl --lat-batches 0" STEPS=12 bash scripts/ab.sh librl_amd_base.so librl_amd.so || exit $?
done
