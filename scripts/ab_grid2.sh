#!/bin/bash
# replay grid on the uniform workloads (RL_COOP_GRID)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for wl in fw_uniform sw_bursty mixed tb_zipf; do
  for g in 96 160 256; do
    RL_COOP_GRID=$g timeout -k 10 200 python bench.py --workload $wl --steps 12 --warmup 3 --no-cpu-baseline --lat-batches 0 2>/dev/null \
      | python -c "import json,sys; d=json.load(sys.stdin); print('$wl grid $g', round(d['value']/1e6,1), {k: round(x,3) for k,x in d['stages_ms_per_batch'].items()})" || exit 1
  done
done
