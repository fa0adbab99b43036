#!/bin/bash
# A/B of engine environment settings on one box: each argument is an env
# assignment list ("-" for none), alternated twice; prints value and stage ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for v in "$@"; do
    envs=""; [ "$v" != "-" ] && envs="$v"
    env $envs timeout -k 10 200 python bench.py --steps ${STEPS:-12} --warmup 2 --no-cpu-baseline ${BARGS:-} \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']/1e6,1), {k: round(x,4) for k,x in d.get('stages_ms_per_batch',{}).items()})" || exit 1
  done
done
