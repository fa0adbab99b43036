#!/bin/bash
# A/B: events bound to dispatch packets (default: replay timing events,
# front_done on k_permute, chain_done on the replay) vs marker packets
# (RL_EV_MARKERS=1), alternating runs on one box; $EXTRA env for both
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2 3; do
  for v in "X=0" "RL_EV_MARKERS=1"; do
    env $v ${EXTRA:-} timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline ${BARGS:-} \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$v ${EXTRA:-}]', round(d['value']/1e6,1), d['roofline']['achieved'], {k: round(x,4) for k,x in d['stages_ms_per_batch'].items()})" || exit 1
  done
done
