#!/bin/bash
# A/B: grouping sort variants -- base (HEAD), scaled MSD digit + rows spread
# over all waves (librl_amd.so), plain digit + rows spread (plain)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for wl in mixed fw_uniform sw_bursty; do
  echo "== $wl"
  BARGS="--workload $wl --lat-batches 0" STEPS=20 bash scripts/ab.sh librl_amd_base.so librl_amd.so librl_amd_plain.so || exit 1
done
