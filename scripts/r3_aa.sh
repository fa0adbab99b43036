#!/bin/bash
# upper bound of dropping the skipped LSD passes / k_segments launches (unsafe A/B: valid only when every MSD bucket fits k_sort_local)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for wl in mixed fw_uniform sw_bursty mixed fw_uniform sw_bursty; do
  for v in 0 1; do
    if [ $v = 1 ]; then export RL_AB_NOLSD=1; else unset RL_AB_NOLSD; fi
    timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 2 --no-cpu-baseline --lat-batches 0 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl nolsd=$v', round(d['value']/1e6,1), {k: round(x,4) for k,x in d['stages_ms_per_batch'].items()})" || exit 1
  done
done
