#!/bin/bash
# kernel traces: mixed routed vs mixed local (timeline comparison)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r3x_routed NO_PMC=1 BARGS="--workload mixed --ingress routed --steps 12 --warmup 2 --no-cpu-baseline --lat-batches 0" bash scripts/profile.sh || exit 1
TAG=r3x_local NO_PMC=1 BARGS="--workload mixed --steps 12 --warmup 2 --no-cpu-baseline --lat-batches 0" bash scripts/profile.sh || exit 1
