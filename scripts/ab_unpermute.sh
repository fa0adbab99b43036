#!/bin/bash
# A/B of the finish stage: bucketed unpermute (default) vs direct scatter
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for w in ${WORKLOADS:-tb_zipf mixed}; do
  TAG="$w bucket " BARGS="--workload $w --lat-batches 0" STEPS=12 bash scripts/bench_brief.sh || exit 1
  RL_SCATTER_UNPERMUTE=1 TAG="$w scatter" BARGS="--workload $w --lat-batches 0" STEPS=12 bash scripts/bench_brief.sh || exit 1
done
