#!/bin/bash
# A/B of engine knobs given as environment assignments, one variant per line
# of $VARIANTS ("" = default), over $WORKLOADS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
while IFS= read -r v; do
  for w in ${WORKLOADS:-tb_zipf mixed}; do
    env $v TAG="$w [$v]" BARGS="--workload $w --lat-batches 0" STEPS=12 bash scripts/bench_brief.sh | cut -c1-190 || exit 1
  done
done <<< "${VARIANTS:-}"
