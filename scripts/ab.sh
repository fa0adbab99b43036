#!/bin/bash
# A/B: alternate bench runs of several engine builds in ONE process-per-run
# sequence on the same box; prints value and replay ms for each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=distributed-rate-limiter_amd/lib
for rep in 1 2; do
  for v in "$@"; do
    RL_AMD_LIB=$PWD/$L/$v timeout -k 10 200 python bench.py --steps ${STEPS:-12} --warmup 2 --no-cpu-baseline ${BARGS:-} \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']/1e6,1), {k: round(x,4) for k,x in d.get('stages_ms_per_batch',{}).items()})" || exit 1
  done
done
