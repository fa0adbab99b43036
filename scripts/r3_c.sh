# configs[4] stall attribution: the load generator under a HIP API trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
rm -rf /tmp/stall
RL_COALESCER_TRACE=65536 timeout -s KILL 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d /tmp/stall -o run -- distributed-rate-limiter_amd/lib/rl_bench_e2e --qps 3e6 --seconds 3 > gpurun_out/r3c_stall_e2e_$i.json 2> gpurun_out/r3c_stall_e2e_$i.err || { tail gpurun_out/r3c_stall_e2e_$i.err; exit 1; }
python scripts/stall_trace.py /tmp/stall gpurun_out/r3c_stall_trace_$i.json
done
