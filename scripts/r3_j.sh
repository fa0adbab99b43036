# routed host-side profile (RL_ROUTE_PROFILE: host seconds per call site)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in 2 4; do
RL_ROUTE_LOOKAHEAD=$L RL_ROUTE_PROFILE=1 timeout -k 10 200 python bench.py --workload mixed --ingress routed --steps 20 --warmup 3 --no-cpu-baseline --lat-batches 0 > gpurun_out/r3j_routed_prof_L$L.json 2> gpurun_out/r3j_routed_prof_L$L.err || { tail gpurun_out/r3j_routed_prof_L$L.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r3j_routed_prof_L$L.json')); print('L=$L', d['value']/1e6, d['ms_per_step'], json.dumps(d['config']['host_ms_per_step']))"
done
