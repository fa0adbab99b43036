# routed pipeline A/B: request-path stream priority, merge stream
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export RL_ROUTE_B_FIRST=1
for cfg in "0 0" "1 0" "1 1" "0 0" "1 0"; do
  set -- $cfg
  if [ "$1" = 1 ]; then export RL_ROUTE_R_PRIO=1; else unset RL_ROUTE_R_PRIO; fi
  if [ "$2" = 1 ]; then export RL_ROUTE_MERGE_ON_R=1; else unset RL_ROUTE_MERGE_ON_R; fi
  timeout -k 10 200 python bench.py --workload mixed --ingress routed --steps 30 --warmup 3 --no-cpu-baseline --lat-batches 0 > gpurun_out/r3k.json 2> gpurun_out/r3k.err || { tail gpurun_out/r3k.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r3k.json')); print('rprio=$1 merge_on_r=$2', round(d['value']/1e6,1), round(d['ms_per_step'],3), json.dumps(d['config']['host_ms_per_step']))"
done
