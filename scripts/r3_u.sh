# configs[1] over more of its 64-batch trace: 20 vs 56 timed steps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for st in 20 56 20 56; do
  s0=$(date +%s.%N)
  timeout -k 10 300 python bench.py --steps $st --warmup 4 --no-cpu-baseline > gpurun_out/r3u_$st.json 2> gpurun_out/r3u_$st.err || { tail gpurun_out/r3u_$st.err; exit 1; }
  s1=$(date +%s.%N)
  python -c "
import json; d=json.load(open('gpurun_out/r3u_$st.json')); print('steps=$st', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), 'ms/step replay', round(d['roofline']['launch_ms'],4), 'p99', round(d['latency']['p99_batch_ms'],3), 'wall', round($s1-$s0,1), 's')"
done
