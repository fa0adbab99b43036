#!/bin/bash
# A/B: probe histograms of the MSD pass only on a predicted plan (librl_amd.so) vs HEAD (base); probe grid 2048 on top
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread -k "predicted or sort_local or config0 or mixed" > gpurun_out/r3ad_tests.txt 2>&1 || { tail -30 gpurun_out/r3ad_tests.txt; exit 1; }
tail -1 gpurun_out/r3ad_tests.txt
for wl in mixed sw_bursty fw_uniform; do
  echo "== $wl"
  BARGS="--workload $wl --lat-batches 0" STEPS=20 bash scripts/ab.sh librl_amd_base.so librl_amd.so || exit 1
  RL_PROBE_GRID=2048 BARGS="--workload $wl --lat-batches 0" STEPS=20 bash scripts/ab.sh librl_amd.so | sed 's/^/grid2048 /' || exit 1
done
