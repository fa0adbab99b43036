#!/bin/bash
# A/B of the replay grid (RL_COOP_GRID): CUs left to the grouping / finish streams
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for w in ${WORKLOADS:-tb_zipf mixed}; do
  for g in ${GRIDS:-512 256 192 128}; do
    RL_COOP_GRID=$g TAG="$w grid=$g" BARGS="--workload $w --lat-batches 0" STEPS=12 bash scripts/bench_brief.sh | cut -c1-200 || exit 1
  done
done
